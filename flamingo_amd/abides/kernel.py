"""Discrete-event simulation kernel (Kernel.py surface).

Single-threaded event loop over a time-ordered heap of WAKEUP and MESSAGE
events (Kernel.py:190-271).  Each agent carries its own clock: after it acts
its clock advances by its computation delay (plus any transient delay it
asked for), and events that reach an agent that is still "in the future" are
re-queued at the agent's clock (Kernel.py:217-223, 246-252).  Messages are
delivered at send time + computation delay + sampled network latency
(Kernel.py:329-394).  Message bodies travel by reference.

API kept from the reference: Kernel(kernel_name, random_state), runner(...)
returning custom_state, sendMessage, setWakeup, get/setAgentComputeDelay,
delayAgent, findAgentByType, writeLog, appendSummaryLog, writeSummaryLog,
updateAgentState, fmtTime.
"""
from __future__ import annotations

import heapq
import itertools
import os

import numpy as np
import pandas as pd

from . import log
from .message import MessageType


class Kernel:
    def __init__(self, kernel_name, random_state=None):
        if not random_state:
            raise ValueError(f"A valid, seeded np.random.RandomState object is required for the Kernel {kernel_name}")
        self.name = kernel_name
        self.random_state = random_state
        self._events = []
        self._seq = itertools.count()
        self.currentTime = None
        self.kernelWallClockStart = pd.Timestamp("now")
        self.meanResultByAgentType = {}
        self.agentCountByType = {}
        self.summaryLog = []
        self.custom_state = {}
        log.log_print("Kernel initialized: {}", self.name)

    # ------------------------------------------------------------ queue
    def _push(self, when, recipient, mtype, msg):
        # Kernel.py orders (time, (recipient, type, msg)): ties go to the lower recipient id, then
        # MESSAGE before WAKEUP, then the message created first (Message.__lt__ on uniq), also
        # when an event is re-queued for an agent that is in the future.
        tie = msg.uniq if msg is not None else next(self._seq)
        heapq.heappush(self._events, (when, recipient, mtype.value, tie, next(self._seq), mtype, msg))

    @property
    def messages(self):
        """Pending events as (time, (recipient, type, msg)) in delivery order (read-only view)."""
        return [(e[0], (e[1], e[5], e[6])) for e in sorted(self._events)]

    # ----------------------------------------------------------- runner
    def runner(self, agents=(), startTime=None, stopTime=None, num_simulations=1, defaultComputationDelay=1,
               defaultLatency=1, agentLatency=None, latencyNoise=(1.0,), agentLatencyModel=None, skip_log=False,
               seed=None, oracle=None, log_dir=None):
        self.agents = list(agents)
        self.custom_state = {}
        self.startTime, self.stopTime = startTime, stopTime
        self.seed, self.skip_log, self.oracle = seed, skip_log, oracle
        self.log_dir = log_dir or str(int(self.kernelWallClockStart.timestamp()))
        n = len(self.agents)
        self.agentCurrentTimes = [startTime] * n
        self.agentComputationDelays = [defaultComputationDelay] * n
        self.agentLatencyModel = agentLatencyModel
        self.agentLatency = agentLatency if agentLatency is not None else [[defaultLatency] * n for _ in range(n)]
        self.latencyNoise = list(latencyNoise)
        self.currentAgentAdditionalDelay = 0
        log.log_print("Kernel started: {}", self.name)

        for sim in range(num_simulations):
            log.log_print("Starting sim {}", sim)
            for a in self.agents:
                a.kernelInitializing(self)
            for a in self.agents:
                a.kernelStarting(self.startTime)
            self.currentTime = self.startTime
            wall0 = pd.Timestamp("now")
            handled = 0
            while self._events and self.currentTime is not None and self.currentTime <= self.stopTime:
                when, recipient, _, _, _, mtype, msg = heapq.heappop(self._events)
                self.currentTime = when
                if handled % 100000 == 0:
                    print(f"\n--- Simulation time: {self.currentTime}, messages processed: {handled}, "
                          f"wallclock elapsed: {pd.Timestamp('now') - wall0} ---\n")
                handled += 1
                self.currentAgentAdditionalDelay = 0
                if self.agentCurrentTimes[recipient] > self.currentTime:
                    # the agent is still busy: deliver when its clock says it is free
                    self._push(self.agentCurrentTimes[recipient], recipient, mtype, msg)
                    continue
                self.agentCurrentTimes[recipient] = self.currentTime
                if mtype == MessageType.WAKEUP:
                    self.agents[recipient].wakeup(self.currentTime)
                elif mtype == MessageType.MESSAGE:
                    self.agents[recipient].receiveMessage(self.currentTime, msg)
                else:
                    raise ValueError("Unknown message type found in queue", self.currentTime, mtype)
                self.agentCurrentTimes[recipient] += pd.Timedelta(
                    self.agentComputationDelays[recipient] + self.currentAgentAdditionalDelay)
            elapsed = pd.Timestamp("now") - wall0
            for a in self.agents:
                a.kernelStopping()
            for a in self.agents:
                a.kernelTerminating()
            secs = max(elapsed / np.timedelta64(1, "s"), 1e-9)
            print(f"Event Queue elapsed: {elapsed}, messages: {handled}, messages per second: {handled / secs:0.1f}")
            log.log_print("Ending sim {}", sim)

        self.custom_state["kernel_event_queue_elapsed_wallclock"] = elapsed
        self.custom_state["kernel_slowest_agent_finish_time"] = max(self.agentCurrentTimes)
        self.writeSummaryLog()
        print("Simulation ending!")
        return self.custom_state

    # ----------------------------------------------------- agent services
    def sendMessage(self, sender=None, recipient=None, msg=None, delay=0, tag=None):
        if sender is None or recipient is None or msg is None:
            raise ValueError("sendMessage() needs sender, recipient and msg", sender, recipient, msg)
        sent = self.currentTime + pd.Timedelta(self.agentComputationDelays[sender] + self.currentAgentAdditionalDelay
                                               + delay)
        if self.agentLatencyModel is not None:
            latency = self.agentLatencyModel.get_latency(sender_id=sender, recipient_id=recipient)
            if tag:
                self.custom_state[tag] = self.custom_state.get(tag, pd.Timedelta(0)) + pd.Timedelta(latency)
        else:
            noise = self.random_state.choice(len(self.latencyNoise), 1, p=self.latencyNoise)[0]
            latency = self.agentLatency[sender][recipient] + noise
        self._push(sent + pd.Timedelta(latency), recipient, MessageType.MESSAGE, msg)

    def setWakeup(self, sender=None, requestedTime=None):
        if sender is None:
            raise ValueError("setWakeup() called without valid sender ID")
        if requestedTime is None:
            requestedTime = self.currentTime + pd.Timedelta(1)
        if self.currentTime is not None and requestedTime < self.currentTime:
            raise ValueError("setWakeup() called with requested time not in future", self.currentTime, requestedTime)
        self._push(requestedTime, sender, MessageType.WAKEUP, None)

    def getAgentComputeDelay(self, sender=None):
        return self.agentComputationDelays[sender]

    def setAgentComputeDelay(self, sender=None, requestedDelay=None):
        if not isinstance(requestedDelay, int):
            raise ValueError("Requested computation delay must be whole nanoseconds.", requestedDelay)
        if requestedDelay < 0:
            raise ValueError("Requested computation delay must be non-negative nanoseconds.", requestedDelay)
        self.agentComputationDelays[sender] = requestedDelay

    def delayAgent(self, sender=None, additionalDelay=None):
        if not isinstance(additionalDelay, int):
            raise ValueError("Additional delay must be whole nanoseconds.", additionalDelay)
        if additionalDelay < 0:
            raise ValueError("Additional delay must be non-negative nanoseconds.", additionalDelay)
        self.currentAgentAdditionalDelay += additionalDelay

    def findAgentByType(self, type=None):
        for a in self.agents:
            if isinstance(a, type):
                return a.id

    # ------------------------------------------------------------- logs
    def _log_path(self):
        path = os.path.join(".", "log", self.log_dir)
        os.makedirs(path, exist_ok=True)
        return path

    def writeLog(self, sender, dfLog, filename=None):
        if self.skip_log:
            return
        name = filename or self.agents[sender].name.replace(" ", "")
        dfLog.to_pickle(os.path.join(self._log_path(), f"{name}.bz2"), compression="bz2")

    def appendSummaryLog(self, sender, eventType, event):
        self.summaryLog.append({"AgentID": sender, "AgentStrategy": self.agents[sender].type,
                                "EventType": eventType, "Event": event})

    def writeSummaryLog(self):
        if self.skip_log:
            return
        pd.DataFrame(self.summaryLog).to_pickle(os.path.join(self._log_path(), "summary_log.bz2"), compression="bz2")

    def updateAgentState(self, agent_id, state):
        self.custom_state.setdefault("agent_state", {})[agent_id] = state

    @staticmethod
    def fmtTime(simulationTime):
        return simulationTime
