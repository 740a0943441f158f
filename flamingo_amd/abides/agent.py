"""Agent base class (agent/Agent.py surface).

Lifecycle hooks called by the Kernel: kernelInitializing -> kernelStarting ->
(wakeup / receiveMessage)* -> kernelStopping -> kernelTerminating
(agent/Agent.py:52-139).  Services go through the kernel by agent id only:
sendMessage, setWakeup, get/setComputationDelay, delay, writeLog,
updateAgentState (:148-173).
"""
from __future__ import annotations

from copy import deepcopy

import pandas as pd

from . import log


class Agent:
    def __init__(self, id, name, type, random_state):
        if not random_state:
            raise ValueError(f"A valid, seeded np.random.RandomState object is required for agent {name}")
        self.id = id
        self.name = name
        self.type = type
        self.random_state = random_state
        self.kernel = None
        self.currentTime = None
        self.log = []
        self.logEvent("AGENT_TYPE", type)

    # ---- lifecycle
    def kernelInitializing(self, kernel):
        self.kernel = kernel
        log.log_print("{} exists!", self.name)

    def kernelStarting(self, startTime):
        log.log_print("Agent {} ({}) requesting kernel wakeup at time {}", self.id, self.name, startTime)
        self.setWakeup(startTime)

    def kernelStopping(self):
        pass

    def kernelTerminating(self):
        if self.log:
            df = pd.DataFrame(self.log)
            df.set_index("EventTime", inplace=True)
            self.writeLog(df)

    # ---- bookkeeping
    def logEvent(self, eventType, event="", appendSummaryLog=False):
        e = deepcopy(event)
        self.log.append({"EventTime": self.currentTime, "EventType": eventType, "Event": e})
        if appendSummaryLog:
            self.kernel.appendSummaryLog(self.id, eventType, e)

    # ---- called by the kernel
    def receiveMessage(self, currentTime, msg):
        self.currentTime = currentTime
        log.log_print("At {}, agent {} ({}) received: {}", currentTime, self.id, self.name, msg)

    def wakeup(self, currentTime):
        self.currentTime = currentTime
        log.log_print("At {}, agent {} ({}) received wakeup.", currentTime, self.id, self.name)

    # ---- kernel services
    def sendMessage(self, recipientID, msg, delay=0, tag="communication"):
        self.kernel.sendMessage(self.id, recipientID, msg, delay=delay, tag=tag)

    def setWakeup(self, requestedTime):
        self.kernel.setWakeup(self.id, requestedTime)

    def getComputationDelay(self):
        return self.kernel.getAgentComputeDelay(sender=self.id)

    def setComputationDelay(self, requestedDelay):
        self.kernel.setAgentComputeDelay(sender=self.id, requestedDelay=requestedDelay)

    def delay(self, additionalDelay):
        self.kernel.delayAgent(sender=self.id, additionalDelay=additionalDelay)

    def writeLog(self, dfLog, filename=None):
        self.kernel.writeLog(self.id, dfLog, filename)

    def updateAgentState(self, state):
        self.kernel.updateAgentState(self.id, state)

    def __lt__(self, other):
        return str(self.id) < str(other.id)
