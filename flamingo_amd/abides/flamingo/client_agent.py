"""Flamingo client agent (agent/flamingo/SA_ClientAgent.py surface).

Per iteration the client (sendVectors, :198-348) finds its neighbours, draws
its self-mask seed m_i, Shamir-shares it to the committee (each share AES-GCM
encrypted under the ECDH key with that member, :214-244), derives a pairwise
seed per neighbour -- ECDH r_ij = a_i A_j -> SHA-256 -> key; h_ijt =
ChaCha20(key)(t) & 0xFFFF; H = hash_to_curve(h_ijt); s_ij = SHA-256(H)
(:253-292) -- ElGamal-encrypts H under the system key (:326-332, :434-447)
and sends the masked vector

    y_i = x_i + PRG(m_i) + sum_{j in N(i), j > i} PRG(s_ij) - sum_{j < i} PRG(s_ij)

(:304-324; x_i = all ones, :304).  GPU work: the mask expansion and
composition (MaskEngine.client_mask) and every batch of P-256 scalar
multiplications (ECDH, ElGamal, decryption shares: MaskEngine.ec_mul_wire).
Committee members sign the offline set (ECDSA, :351-368) and answer DEC with
sk_j * c0 for each dropout ciphertext plus their decrypted m_i shares
(:370-431).
"""
from __future__ import annotations

import logging

import numpy as np
import pandas as pd

from ... import crypto as C
from ..agent import Agent
from ..message import Message
from . import protocol as param
from . import wire
from .seeds import P256_N, shamir_share
from .service_agent import SA_ServiceAgent as ServiceAgent

_MASK128 = (1 << 128) - 1



def pair_prf(engine, keys, iteration: int) -> list:
    """h_ijt for every pair key r_ij, as the decimal strings the client hashes to the curve
    (SA_ClientAgent.py:276-283): str(int.from_bytes(ChaCha20(r_ij, nonce).encrypt(t.to_bytes(16,
    'big'))[0:4], 'big') & 0xFFFF).  Bytes 0-3 of that ciphertext are keystream word 0 XOR t's
    first four bytes, so one batched GPU PRG call over all keys gives them: PRG word 0 of a key is
    LE32(keystream[0:4]) ^ "abcd" (util/param.py:12,32)."""
    if not keys:
        return []
    rnd = int(iteration).to_bytes(16, "big")[:4]
    w = np.asarray(engine.prg_expand(list(keys), 1))[:, 0].astype(np.uint32) ^ np.uint32(0x64636261)
    # ciphertext byte k = keystream byte k (LE byte k of word 0) ^ rnd[k]; h = bytes 2..3, big endian
    b2 = ((w >> np.uint32(16)) & np.uint32(0xFF)) ^ np.uint32(rnd[2])
    b3 = ((w >> np.uint32(24)) & np.uint32(0xFF)) ^ np.uint32(rnd[3])
    return [str(v) for v in ((b2 << np.uint32(8)) | b3).tolist()]

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
        pki = param.pki(num_clients)
        self.secret_key = pki.client_sk[id]
        self.public_key = pki.client_pk[id]
        self.system_pk = pki.system_pk
        self.committee_keys = {}     # member -> AES key (a_i A_c).x mod 2^128 (:234-236)
        self.symmetric_keys = {}     # (committee members) client -> AES key (:86-91)
        param.register_client(self)
        if id in self.user_committee:
            ids = list(range(num_clients))
            self.symmetric_keys = self._aes_keys(ids)

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
                    self.decryptSendShares(b["dec_target_pairwise"], b["dec_target_mi"], b["client_id_list"])
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
    def _aes_keys(self, ids) -> dict:
        """(a_i A_j).x mod 2^128 per client j (:234-236, :86-91); the ECDH points of every
        client x committee pair come from one GPU batch (protocol.prefetch_committee_ecdh)."""
        param.prefetch_committee_ecdh(self.num_clients)
        return {j: (int.from_bytes(param.ecdh_wire(self.num_clients, self.id, j)[:32], "big") & _MASK128)
                .to_bytes(16, "big") for j in ids}

    def _rand_scalar(self) -> int:
        return int.from_bytes(bytes(self.random_state.randint(0, 256, size=32, dtype=np.uint8)), "big") % P256_N

    def sendVectors(self, currentTime):
        if self.current_iteration in self.offline_iterations:
            self.logger.info(f"client {self.id} is offline in iteration {self.current_iteration}")
            return
        self.neighbors_list = param.find_neighbors(param.root_seed, self.current_iteration, self.num_clients,
                                                   self.id, self.neighborhood_size)
        nb = list(self.neighbors_list)          # the reference's set order (:256, :295, :330)
        if self.id in self.neighbors_list:
            raise RuntimeError("id itself appears in its neighbor list")
        committee = sorted(self.user_committee)
        # the ECDH keys r_ij = SHA-256(a_i A_j) of the whole iteration's graph: one GPU batch, cached in
        # the protocol (pair_material below)
        if not self.committee_keys:
            self.committee_keys = self._aes_keys(committee)

        # m_i, its Shamir shares, one AES-GCM ciphertext per committee member (:214-244)
        mi_bytes = bytes(self.random_state.randint(0, 256, size=self.key_length, dtype=np.uint8))
        mi_number = int.from_bytes(mi_bytes, "big")
        threshold = int(param.fraction * len(self.user_committee))
        shares = shamir_share(mi_number, max(1, threshold), len(committee), self.prime,
                              rng=_PyRandom(self.random_state))
        enc_mi_shares = []
        for (_, y), cid in zip(shares, committee):
            nonce = bytes(self.random_state.randint(0, 256, size=16, dtype=np.uint8))
            ct, _ = C.aes_gcm_encrypt(self.committee_keys[cid], y.to_bytes(self.key_length, "big"), nonce)
            enc_mi_shares.append((ct, nonce))

        # pairwise seeds: h_ijt -> H (group element) -> s_ij (:266-292), every client's in a few
        # batched launches (protocol.pair_material: one PRG launch for all h_ijt, the hash-to-curve table)
        pnb, _, _, s_ij = param.pair_material(self.current_iteration, self.num_clients,
                                              self.neighborhood_size)[self.id]
        if pnb != nb:
            raise RuntimeError("pair material built for another neighbour order")
        seeds = [mi_bytes] + [s[: self.key_length] for s in s_ij]
        signs = [1] + [1 if self.id < j else -1 for j in nb]

        # ElGamal under the system key: c0 = rG, c1 = H + r pk (:326-332, :434-447); every client's
        # r G and H + r pk of the iteration come from two GPU launches (protocol.elgamal_masks)
        _, rg, c1w = param.elgamal_masks(self, self.current_iteration, nb)
        c0 = C.points_from_wire(rg) if nb else []
        c1 = C.points_from_wire(c1w) if nb else []
        cipher = {(self.id, j): (c0[k], c1[k]) for k, j in enumerate(nb)}

        x = None if self.input_vector is None else np.asarray(self.input_vector, np.uint32)[None, :]
        vec = param.engine().client_mask(np.array([0, len(seeds)], np.int64), seeds, signs, self.vector_len, x=x)[0]
        self.sendMessage(self.serviceAgentID, Message({
            "msg": "VECTOR", "iteration": self.current_iteration, "sender": self.id, "vector": vec,
            "enc_mi_shares": wire.serialize_tuples_bytes(enc_mi_shares),
            "enc_pairwise": wire.serialize_dim1_elgamal(cipher)}),
            tag="comm_key_generation")

    def signSendLabels(self, currentTime, msg_to_sign):
        payload = repr(msg_to_sign).encode()          # the reference signs dill.dumps(msg) (:352-356)
        sig = C.ecdsa_sign(self.secret_key, self.public_key, payload)
        self.sendMessage(self.serviceAgentID, Message({
            "msg": "SIGN", "iteration": self.current_iteration, "sender": self.id,
            "signed_labels": (payload, sig), "committee_member_idx": self.committee_member_idx}),
            tag="comm_sign_client")

    def decryptSendShares(self, dec_target_pairwise, dec_target_mi, client_id_list):
        """dec_target_pairwise: serialize_dim1_elgamal JSON; dec_target_mi: serialize_tuples_bytes JSON."""
        if self.committee_shared_sk is None:
            self.sendMessage(self.serviceAgentID, Message({
                "msg": "NO_SK_SHARE", "iteration": self.current_iteration, "sender": self.id,
                "shared_result": None, "committee_member_idx": None}), tag="no_sk_share")
            return
        # sk_j * c0 for every dropout ciphertext (:393-400), one GPU batch
        _, c0w, _ = wire.elgamal_json_to_wire(dec_target_pairwise)
        sk = self.committee_shared_sk[1]
        dec_w, _ = param.engine().ec_mul_wire(c0w, C.scalars_to_wire([sk] * c0w.shape[0]))
        # decrypt this member's m_i shares (:402-420)
        dec_mi = []
        for cid, (ct, nonce) in zip(client_id_list, wire.deserialize_tuples_bytes(dec_target_mi)):
            dec_mi.append(int.from_bytes(C.aes_gcm_decrypt(self.symmetric_keys[cid], ct, nonce), "big"))
        self.sendMessage(self.serviceAgentID, Message({
            "msg": "SHARED_RESULT", "iteration": self.current_iteration, "sender": self.id,
            "shared_result_pairwise": wire.wire_to_ecp_json(dec_w),
            "shared_result_mi": wire.serialize_dim1_list(dec_mi),
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
