"""Flamingo client agent (agent/flamingo/SA_ClientAgent.py surface).

Per iteration the client (sendVectors, :198-348) finds its neighbours, draws
its self-mask seed m_i, deals Shamir shares of m_i to the committee, derives a
pairwise seed per neighbour and sends the masked vector

    y_i = x_i + PRG(m_i) + sum_{j in N(i), j > i} PRG(s_ij) - sum_{j < i} PRG(s_ij)

(:304-324; x_i = all ones, :304).  The mask expansion and composition run on
the GPU (MaskEngine.client_mask).  Committee members answer the server's SIGN
and DEC requests (signSendLabels :351-368, decryptSendShares :370-431).
Crypto stand-ins: see seeds.py.
"""
from __future__ import annotations

import hashlib
import json
import logging

import numpy as np
import pandas as pd

from ..agent import Agent
from ..message import Message
from . import protocol as param
from .seeds import P256_N, pair_seed, shamir_share
from .service_agent import SA_ServiceAgent as ServiceAgent


class SA_ClientAgent(Agent):
    def __str__(self):
        return "[client]"

    def __init__(self, id, name, type, iterations=4, key_length=32, num_clients=128, neighborhood_size=1,
                 debug_mode=0, random_state=None, offline_iterations=()):
        super().__init__(id, name, type, random_state)
        self.logger = logging.getLogger(__name__)
        self.logger.setLevel(logging.INFO)
        if debug_mode:
            logging.basicConfig()
        self.num_clients = num_clients
        self.neighborhood_size = neighborhood_size
        self.vector_len = param.vector_len
        self.vector_dtype = param.vector_type
        self.prime = P256_N
        self.key_length = key_length
        self.neighbors_list = set()
        self.cipher_stored = None
        self.user_committee = param.committee(self.num_clients)
        self.committee_shared_sk = None
        self.committee_member_idx = None
        self.elapsed_time = {"REPORT": pd.Timedelta(0), "CROSSCHECK": pd.Timedelta(0),
                             "RECONSTRUCTION": pd.Timedelta(0)}
        self.no_of_iterations = iterations
        self.current_iteration = 1
        self.current_base = 0
        self.setup_complete = False
        # iterations in which this client crashes before sending (explicit dropout injection;
        # in the reference dropouts only come from late messages)
        self.offline_iterations = set(offline_iterations)
        self.input_vector = None     # None -> all ones (:304)

    def kernelStarting(self, startTime):
        if self.id == 0:
            for k in ("clt_report", "clt_crosscheck", "clt_reconstruction"):
                self.kernel.custom_state[k] = pd.Timedelta(0)
        self.serviceAgentID = self.kernel.findAgentByType(ServiceAgent)
        self.setComputationDelay(0)
        super().kernelStarting(startTime + pd.Timedelta(self.random_state.randint(low=0, high=1000), unit="ns"))

    def kernelStopping(self):
        for k, cat in (("clt_report", "REPORT"), ("clt_crosscheck", "CROSSCHECK"),
                       ("clt_reconstruction", "RECONSTRUCTION")):
            self.kernel.custom_state[k] = self.kernel.custom_state.get(k, pd.Timedelta(0)) + \
                self.elapsed_time[cat] / self.no_of_iterations
        super().kernelStopping()

    def wakeup(self, currentTime):
        super().wakeup(currentTime)
        self.sendVectors(currentTime)

    def receiveMessage(self, currentTime, msg):
        super().receiveMessage(currentTime, msg)
        body = msg.body
        if body["msg"] == "COMMITTEE_SHARED_SK":
            self.committee_shared_sk = body["sk_share"]
            self.committee_member_idx = body["committee_member_idx"]
        elif body["msg"] == "SIGN":
            if body["iteration"] == self.current_iteration:
                t0 = pd.Timestamp("now")
                self.cipher_stored = msg
                self.signSendLabels(currentTime, body["labels"])
                self.recordTime(t0, "CROSSCHECK")
        elif body["msg"] == "DEC":
            if body["iteration"] == self.current_iteration:
                t0 = pd.Timestamp("now")
                if self.cipher_stored is not None and self.cipher_stored.body["iteration"] == self.current_iteration:
                    b = self.cipher_stored.body
                    self.decryptSendShares(json.loads(b["dec_target_pairwise"]), json.loads(b["dec_target_mi"]),
                                           b["client_id_list"])
                self.cipher_stored = None
                self.recordTime(t0, "RECONSTRUCTION")
        elif body["msg"] == "REQ" and self.current_iteration != 0:
            self.current_iteration += 1
            if self.current_iteration > self.no_of_iterations:
                return
            t0 = pd.Timestamp("now")
            self.sendVectors(currentTime)
            self.recordTime(t0, "REPORT")

    # --------------------------------------------------------------- round
    def sendVectors(self, currentTime):
        if self.current_iteration in self.offline_iterations:
            self.logger.info(f"client {self.id} is offline in iteration {self.current_iteration}")
            return
        self.neighbors_list = param.find_neighbors(param.root_seed, self.current_iteration, self.num_clients,
                                                   self.id, self.neighborhood_size)
        mi_bytes = bytes(self.random_state.randint(0, 256, size=self.key_length, dtype=np.uint8))
        mi_number = int.from_bytes(mi_bytes, "big")
        threshold = int(param.fraction * len(self.user_committee))
        shares = shamir_share(mi_number, max(1, threshold), len(self.user_committee), self.prime,
                              rng=_PyRandom(self.random_state))
        enc_mi_shares = [y for _, y in shares]           # AES-GCM stand-in: share values in the clear
        seeds = [mi_bytes]
        signs = [1]
        pairwise = {}
        for j in sorted(self.neighbors_list):
            if j == self.id:
                raise RuntimeError("id itself appears in its neighbor list")
            s = pair_seed(param.root_seed, self.current_iteration, self.id, j)
            seeds.append(s)
            signs.append(1 if self.id < j else -1)
            pairwise[json.dumps([self.id, j])] = s.hex()   # ElGamal stand-in
        x = None if self.input_vector is None else np.asarray(self.input_vector, np.uint32)[None, :]
        vec = param.engine().client_mask(np.array([0, len(seeds)], np.int64), seeds, signs, self.vector_len, x=x)[0]
        self.sendMessage(self.serviceAgentID, Message({
            "msg": "VECTOR", "iteration": self.current_iteration, "sender": self.id, "vector": vec,
            "enc_mi_shares": json.dumps(enc_mi_shares), "enc_pairwise": json.dumps(pairwise)}),
            tag="comm_key_generation")

    def signSendLabels(self, currentTime, msg_to_sign):
        labels, _ = msg_to_sign
        sig = hashlib.sha256(b"%d" % self.id + labels.encode()).hexdigest()   # DSS stand-in
        self.sendMessage(self.serviceAgentID, Message({
            "msg": "SIGN", "iteration": self.current_iteration, "sender": self.id,
            "signed_labels": (labels, sig), "committee_member_idx": self.committee_member_idx}),
            tag="comm_sign_client")

    def decryptSendShares(self, dec_target_pairwise, dec_target_mi, client_id_list):
        if self.committee_shared_sk is None:
            self.sendMessage(self.serviceAgentID, Message({
                "msg": "NO_SK_SHARE", "iteration": self.current_iteration, "sender": self.id,
                "shared_result": None, "committee_member_idx": None}), tag="no_sk_share")
            return
        self.sendMessage(self.serviceAgentID, Message({
            "msg": "SHARED_RESULT", "iteration": self.current_iteration, "sender": self.id,
            "shared_result_pairwise": json.dumps(dec_target_pairwise),
            "shared_result_mi": json.dumps(dec_target_mi),
            "committee_member_idx": self.committee_member_idx}), tag="comm_secret_sharing")

    def recordTime(self, startTime, categoryName):
        self.elapsed_time[categoryName] += pd.Timestamp("now") - startTime

    def agent_print(*args, **kwargs):
        print(*args, **kwargs)


class _PyRandom:
    """randrange() over a numpy RandomState, so share polynomials follow the agent's seed."""

    def __init__(self, rs):
        self.rs = rs

    def randrange(self, n):
        return int.from_bytes(bytes(self.rs.randint(0, 256, size=40, dtype=np.uint8)), "big") % n
