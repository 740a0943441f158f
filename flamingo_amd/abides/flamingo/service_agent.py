"""Flamingo server agent (agent/flamingo/SA_ServiceAgent.py surface).

Four-step round state machine, same as the reference (:123-135):
  0 initialize          choose committee, deal the decryption-key shares
  1 report              collect VECTORs; partial sum S; dropout pairs + signs
  2 forward_signatures  forward the committee's signed offline set (DEC)
  3 reconstruction      recover m_i from committee shares; unmask; combine

The hot loops are replaced by calls into the MI355X engine (protocol.server_engine(): the one
MaskEngine, or a DeviceGroup over several GPUs when FLM_GPUS / FLM_GROUP_DEVICES ask for it),
with the vectors device-resident from arrival to the final sum (flamingo_amd.ingest.VectorStore):
  receiveMessage VECTOR store y_i on arrival     (:205-210)  -> VectorStore.add (async H2D, pinned ring)
  report_process        S = sum_{i in U} y_i      (:346-350)  -> VectorStore.partial_sum (S stays on device)
  reconstruction_process
      s_ij for dropout pairs: c1 - sum_j lambda_j (sk_j c0), SHA-256   (:542-585) -> MaskEngine.ec_combine_wire
      out = S - sum PRG(m_i) + sum sigma PRG(s_ij)  (:529-540, :587-605) -> VectorStore.unmask(seeds, signs)
      m_i for online clients: sum_j lambda_j y_{j,i} mod n      (:506-526) -> MaskEngine.shamir_combine
The vector arithmetic is bit-exact with the reference's numpy uint32 code.
Message payloads use the reference's JSON formats (wire.py).
"""
from __future__ import annotations

import json
import logging

import numpy as np
import pandas as pd

from ... import crypto as C
from ... import params as P
from ..agent import Agent
from ..message import Message
from . import protocol as param
from . import wire
from .seeds import P256_N, lagrange_at_zero, shamir_share


class SA_ServiceAgent(Agent):
    def __str__(self):
        return "[server]"

    def __init__(self, id, name, type, random_state=None, msg_fwd_delay=1000000, round_time=pd.Timedelta("10s"),
                 iterations=4, key_length=32, num_clients=10, neighborhood_size=1, parallel_mode=1, debug_mode=0,
                 users={}):
        super().__init__(id, name, type, random_state)
        self.logger = logging.getLogger(__name__)
        self.logger.setLevel(logging.INFO)
        if debug_mode:
            logging.basicConfig()
        self.msg_fwd_delay = msg_fwd_delay
        self.round_time = round_time
        self.no_of_iterations = iterations
        self.parallel_mode = parallel_mode
        self.num_clients = num_clients
        self.users = users
        self.vector_len = param.vector_len
        self.vector_dtype = param.vector_type
        self._store = None           # VectorStore: the VECTOR bodies on the GPU(s), from arrival on
        self._accepting = True       # False between report and the end of reconstruction (:488-497)
        self._host_partial = np.zeros(self.vector_len, dtype=self.vector_dtype)
        self.gpu_ms = {}             # iteration -> {"report": ms, "reconstruction": ms} (device time)
        self.final_sum = np.zeros(self.vector_len, dtype=self.vector_dtype)
        self.prime = P256_N
        self.key_length = key_length
        self.neighborhood_size = neighborhood_size
        self.committee_threshold = 0
        self.elapsed_time = {"REPORT": pd.Timedelta(0), "CROSSCHECK": pd.Timedelta(0),
                             "RECONSTRUCTION": pd.Timedelta(0)}
        self.user_vectors, self.pairwise_cipher, self.mi_cipher, self.recon_index = {}, {}, {}, {}
        self.recv_user_vectors, self.recv_pairwise_cipher, self.recv_mi_cipher, self.recv_recon_index = {}, {}, {}, {}
        self.user_committee = set()
        self.committee_shares_pairwise, self.committee_shares_mi, self.committee_sigs = {}, {}, {}
        self.recv_committee_shares_pairwise, self.recv_committee_shares_mi, self.recv_committee_sigs = {}, {}, {}
        self.dec_target_pairwise, self.recon_symbol = {}, {}
        self.current_iteration = 1
        self.current_round = 0
        self.results = {}            # iteration -> final_sum (kept for inspection / tests)
        self.online_counts = {}      # iteration -> |U|
        self.pairs_per_iteration = {}  # iteration -> D dropout pairs recovered
        self.aggProcessingMap = {0: self.initialize, 1: self.report, 2: self.forward_signatures,
                                 3: self.reconstruction}
        self.namedict = {0: "initialize", 1: "report", 2: "forward_signatures", 3: "reconstruction"}

    # ------------------------------------------------------------ lifecycle
    def kernelStarting(self, startTime):
        for k in ("srv_report", "srv_crosscheck", "srv_reconstruction"):
            self.kernel.custom_state[k] = pd.Timedelta(0)
        self.setComputationDelay(0)
        super().kernelStarting(startTime)

    def kernelStopping(self):
        for k, cat in (("srv_report", "REPORT"), ("srv_crosscheck", "CROSSCHECK"),
                       ("srv_reconstruction", "RECONSTRUCTION")):
            self.kernel.custom_state[k] += self.elapsed_time[cat] / self.no_of_iterations
        super().kernelStopping()

    def wakeup(self, currentTime):
        super().wakeup(currentTime)
        self.agent_print(f"wakeup in iteration {self.current_iteration} at function "
                         f"{self.namedict[self.current_round]}; current time is {currentTime}")
        self.aggProcessingMap[self.current_round](currentTime)

    def receiveMessage(self, currentTime, msg):
        super().receiveMessage(currentTime, msg)
        body = msg.body
        sender = body["sender"]
        late = body.get("iteration") != self.current_iteration
        if body["msg"] == "VECTOR":
            if late:
                self.logger.info(f"LATE MSG: VECTOR from iteration {body['iteration']} client {sender}")
                return
            self.recv_user_vectors[sender] = body["vector"]
            if self._accepting:
                self.store().add(sender, body["vector"])        # upload now, overlapping the DES
            self.recv_mi_cipher[sender] = wire.deserialize_tuples_bytes(body["enc_mi_shares"])
            self.recv_pairwise_cipher.update(wire.deserialize_dim1_elgamal(body["enc_pairwise"]))
        elif body["msg"] == "SIGN":
            if not late:
                self.recv_committee_sigs[sender] = body["signed_labels"]
        elif body["msg"] == "SHARED_RESULT":
            if late:
                self.logger.info(f"LATE MSG: SHARED_RESULT from iteration {body['iteration']} client {sender}")
                return
            # pairwise shares stay JSON until reconstruction parses them straight into GPU wire rows
            self.recv_committee_shares_pairwise[sender] = body["shared_result_pairwise"]
            self.recv_committee_shares_mi[sender] = wire.deserialize_dim1_list(body["shared_result_mi"])
            self.recv_recon_index[sender] = body["committee_member_idx"]

    # ------------------------------------------------------- device state
    def store(self):
        if self._store is None:
            self._store = param.vector_store(self.vector_len, max(1, len(self.users) or self.num_clients))
        return self._store

    @property
    def vec_sum_partial(self) -> np.ndarray:
        """S on the host (copied on demand: the round keeps it on the device between report and
        reconstruction, :346-350 -> :605); zeros before the iteration's report, as the reference's
        attribute reads after its reset (:488-497)."""
        if self._store is not None and getattr(self._store, "has_partial", False):
            return self._store.host_partial()
        return self._host_partial

    @vec_sum_partial.setter
    def vec_sum_partial(self, value):
        """Reference-style assignment (e.g. `server.vec_sum_partial = np.zeros(L, uint32)` before
        reconstruction_process, as the reference's attribute allows): without a report this
        iteration, reconstruction_process adds the masks to this value (MaskEngine.mask_accumulate)."""
        if self._store is not None and getattr(self._store, "has_partial", False):
            raise RuntimeError("vec_sum_partial is device-resident after report; assign it before report "
                               "or after the iteration's reset")
        v = np.asarray(value)
        if v.shape != (self.vector_len,):
            raise RuntimeError("Client sends vector of incorrect length.")   # the guard of :348-349
        self._host_partial = np.ascontiguousarray(v, dtype=self.vector_dtype)

    # ---------------------------------------------------------------- round
    def initialize(self, currentTime):
        t0 = pd.Timestamp("now")
        self.user_committee = param.committee(self.num_clients)
        self.committee_threshold = int(param.fraction * len(self.user_committee))
        # Shamir shares of the system decryption key for the committee (:261-279)
        pki = param.pki(self.num_clients)
        shares = shamir_share(pki.system_sk, max(1, self.committee_threshold), len(self.user_committee),
                              self.prime, rng=None)
        for cnt, cid in enumerate(sorted(self.user_committee)):
            self.sendMessage(cid, Message({"msg": "COMMITTEE_SHARED_SK", "sender": self.id,
                                           "committee_member_idx": cnt + 1, "sk_share": shares[cnt]}),
                             tag="comm_dec_server")
        self.current_round = 1
        self.setWakeup(currentTime + (pd.Timestamp("now") - t0) + pd.Timedelta("2s"))

    def report(self, currentTime):
        t0 = pd.Timestamp("now")
        self.report_read_from_pool()
        self.report_process()
        self.report_clear_pool()
        self.report_send_message()
        delay = pd.Timestamp("now") - t0
        self.agent_print("run time for report step:", delay)
        self.recordTime(t0, "REPORT")
        self.current_round = 2
        self.setWakeup(currentTime + delay + pd.Timedelta(P.wt_flamingo_crosscheck_ns))

    def report_read_from_pool(self):
        self.user_vectors, self.recv_user_vectors = self.recv_user_vectors, {}
        self.mi_cipher, self.recv_mi_cipher = self.recv_mi_cipher, {}
        self.pairwise_cipher, self.recv_pairwise_cipher = self.recv_pairwise_cipher, {}

    def report_clear_pool(self):
        self.recv_committee_shares_mi, self.recv_committee_shares_pairwise = {}, {}
        self.recv_recon_index, self.recv_committee_sigs = {}, {}

    def report_process(self):
        self.agent_print("number of collected vectors:", len(self.user_vectors))
        self.client_id_list = list(self.mi_cipher.keys())
        online = set(self.user_vectors.keys())
        offline = set(self.users) - online
        # partial sum on the GPU(s) over the rows uploaded at arrival (:346-350); the length guard
        # of :348-349 raises inside partial_sum.  S stays device-resident until reconstruction.
        st = self.store()
        self._accepting = False
        if st.bad:
            raise RuntimeError("Client sends vector of incorrect length.")
        if len(st) != len(self.user_vectors):
            raise RuntimeError("stored vectors do not match the received ones")
        t0 = pd.Timestamp("now")
        st.partial_sum()
        t1 = pd.Timestamp("now")
        gpu = st.wait_partial()
        self.gpu_ms.setdefault(self.current_iteration, {})["report"] = gpu
        self.agent_print(f"report partial sum: host enqueue {(t1 - t0).total_seconds() * 1e3:.3f} ms, "
                         f"GPU {gpu:.3f} ms ({len(st)} rows on {st.G} device(s), uploaded at arrival)")
        # dropout pairs (online nb, offline id) and their signs (:359-380)
        nbrs = param.neighbors(self.current_iteration, self.num_clients, self.neighborhood_size)
        pairs, signs = P.dropout_pairs(nbrs, online, offline)
        self.dec_target_pairwise, self.recon_symbol = {}, {}
        for pr, sg in zip(pairs, signs):
            if pr not in self.pairwise_cipher:
                raise RuntimeError("Message lost:", pr)
            self.dec_target_pairwise[pr] = self.pairwise_cipher[pr]
            self.recon_symbol[pr] = sg
        # the server signs the offline set (:382-386)
        labels = json.dumps(sorted(offline)).encode()
        pki = param.pki(self.num_clients)
        self.labels_and_sig = (labels, C.ecdsa_sign(pki.server_sk, pki.server_pk, labels))

    def report_send_message(self):
        # the pairwise ciphertexts are the same JSON for every committee member: serialised once
        # (the reference re-serialises them per member inside this loop, :389-401, line 395)
        pairwise = wire.serialize_dim1_elgamal(self.dec_target_pairwise)
        for cnt, cid in enumerate(sorted(self.user_committee)):
            self.sendMessage(cid, Message({
                "msg": "SIGN", "sender": self.id, "iteration": self.current_iteration,
                "dec_target_pairwise": pairwise,
                "dec_target_mi": wire.serialize_tuples_bytes([self.mi_cipher[c][cnt] for c in self.client_id_list]),
                "client_id_list": self.client_id_list, "labels": self.labels_and_sig}), tag="comm_dec_server")

    def forward_signatures(self, currentTime):
        t0 = pd.Timestamp("now")
        self.committee_sigs = self.recv_committee_sigs
        self.recv_committee_shares_mi = {}
        self.recv_committee_shares_pairwise, self.recv_recon_index = {}, {}
        for cid in sorted(self.user_committee):
            self.sendMessage(cid, Message({"msg": "DEC", "sender": self.id, "iteration": self.current_iteration,
                                           "labels": self.committee_sigs}), tag="comm_sign_server")
        self.current_round = 3
        delay = pd.Timestamp("now") - t0
        self.agent_print("run time for crosscheck step:", delay)
        self.setWakeup(currentTime + delay + pd.Timedelta(P.wt_flamingo_reconstruction_ns))
        self.recordTime(t0, "CROSSCHECK")

    def reconstruction(self, currentTime):
        t0 = pd.Timestamp("now")
        self.committee_shares_pairwise, self.recv_committee_shares_pairwise = self.recv_committee_shares_pairwise, {}
        self.committee_shares_mi, self.recv_committee_shares_mi = self.recv_committee_shares_mi, {}
        self.recon_index, self.recv_recon_index = self.recv_recon_index, {}
        self.reconstruction_process()
        self.reconstruction_clear_pool()
        for uid in self.users:
            self.sendMessage(uid, Message({"msg": "REQ", "sender": 0, "output": 1}), tag="comm_output_server")
        delay = pd.Timestamp("now") - t0
        self.agent_print("run time for reconstruction step:", delay)
        self.recordTime(t0, "RECONSTRUCTION")
        print()
        print("######## Iteration completion ########")
        print(f"[Server] finished iteration {self.current_iteration} at {currentTime + delay}")
        print()
        self.current_round = 1
        self.current_iteration += 1
        if self.current_iteration > self.no_of_iterations:
            return
        self.setWakeup(currentTime + delay + pd.Timedelta(P.wt_flamingo_report_ns))

    def reconstruction_clear_pool(self):
        # (:488-497) late messages of this iteration must not leak into the next one
        self.user_vectors = {}
        self.committee_shares_pairwise, self.committee_shares_mi, self.recon_index = {}, {}, {}
        self.recv_pairwise_cipher, self.recv_mi_cipher, self.recv_user_vectors = {}, {}, {}
        if self._store is not None:
            self._store.reset()
            # the server's devices may have changed (FLM_GPUS / FLM_GROUP_DEVICES / FLM_GROUP_RCCL):
            # a store on the old engine is closed here, between iterations, and made anew on arrival
            if getattr(self._store, "_owner", None) is not None and self._store._owner is not param.server_engine():
                self._store.close()
                self._store = None
        self._host_partial = np.zeros(self.vector_len, dtype=self.vector_dtype)
        self._accepting = True

    def reconstruction_process(self):
        self.agent_print("number of collected shares from decryptors:", len(self.committee_shares_mi))
        if len(self.committee_shares_mi) < self.committee_threshold:
            raise RuntimeError("No enough shares for decryption received.")
        # m_i from the first `threshold` decryptors' shares (:506-526)
        members = list(self.committee_shares_mi.keys())[: max(1, self.committee_threshold)]
        xs = [self.recon_index[m] for m in members]
        coeff = lagrange_at_zero(xs, self.prime)
        # m_i = sum_j lambda_j y_{j,i} mod n for every online client, one GPU batch (T x |U|)
        seeds = param.engine().shamir_combine([self.committee_shares_mi[m] for m in members], coeff)
        signs = [-1] * len(seeds)
        if not self.dec_target_pairwise:
            self.agent_print("no client dropped out.")
        else:
            # threshold ElGamal decryption of every dropout pair's H, then s = SHA-256(H) (:542-585):
            # one GPU batch over D pairs x T decryptors
            c1 = [ct[1] for ct in self.dec_target_pairwise.values()]
            shares = np.stack([wire.ecp_json_to_wire(self.committee_shares_pairwise[m]) for m in members])
            if shares.shape[1] != len(c1):
                raise RuntimeError("length error.")
            _, pair_seeds, flags = param.engine().ec_combine_wire(C.points_to_wire(c1), shares,
                                                                  C.scalars_to_wire(coeff))
            if len(pair_seeds) != len(self.recon_symbol):
                raise RuntimeError("The decrypted length is wrong.")
            for s, sg in zip(pair_seeds, self.recon_symbol.values()):
                seeds.append(bytes(s[: self.key_length]))
                signs.append(sg)
        # final_sum = partial + cancel + mi  (:538-540, :605), on the GPU(s): every device adds the
        # K masks over its own slot shard of the device-resident S, then the one copy to the host
        t0 = pd.Timestamp("now")
        st = self.store()
        if getattr(st, "has_partial", True):
            self.final_sum = st.unmask(seeds, signs)
        else:
            # no report this iteration: the reference-style assigned partial sum (vec_sum_partial
            # setter, :540/:605) is the S the masks are added to, on the GPU
            self.final_sum = param.engine().mask_accumulate(seeds, signs, self._host_partial.copy())
        ms = (pd.Timestamp("now") - t0).total_seconds() * 1e3
        rec = self.gpu_ms.setdefault(self.current_iteration, {})
        rec["reconstruction_unmask_wall"] = ms
        gpu = st.unmask_ms() if hasattr(st, "unmask_ms") and getattr(st, "has_partial", False) else None
        if gpu is not None:
            rec["reconstruction_unmask_gpu"] = gpu
        self.agent_print(f"reconstruction unmask: {len(seeds)} masks over S on the GPU(s) + D2H, {ms:.3f} ms wall"
                         + (f", {gpu:.3f} ms GPU" if gpu is not None else ""))
        self.results[self.current_iteration] = self.final_sum
        self.online_counts[self.current_iteration] = len(self.user_vectors)
        self.pairs_per_iteration[self.current_iteration] = len(self.recon_symbol)
        self.agent_print("final sum:", self.final_sum)

    # ----------------------------------------------------------------- util
    def recordTime(self, startTime, categoryName):
        self.elapsed_time[categoryName] += pd.Timestamp("now") - startTime

    def agent_print(*args, **kwargs):
        print(*args, **kwargs)
