"""Golden fixtures produced BY THE REFERENCE'S OWN CODE (run in the build container only).

Imports, read-only from /root/reference, util/param.py, util/util.py,
util/crypto/{ecchash,secretsharing}, agent/flamingo/SA_ClientAgent.py and
agent/flamingo/SA_ServiceAgent.py, with the absent third-party modules
(pycryptodomex, libnum, utilitybelt) replaced by tests/golden/refshim.py
(OpenSSL-backed ChaCha20 / AES-GCM / P-256, hashlib SHA-256; see its header
for what each stand-in is).  It then drives whole protocol iterations through
the reference agents' own methods, in protocol order:

  SA_ServiceAgent.initialize                          (:252-283)  Shamir of the system sk
  SA_ClientAgent.sendVectors                          (:198-348)  m_i, ECDH, h_ijt, hash-to-curve,
                                                                  PRG composition, ElGamal, AES-GCM
  SA_ServiceAgent.receiveMessage / report             (:188-386)  partial sum, dropout pairs
  SA_ClientAgent.signSendLabels / decryptSendShares   (:351-431)
  SA_ServiceAgent.forward_signatures / reconstruction_process (:403-605)

No kernel event loop: a stub kernel queues each message and this script
delivers them in protocol order (VECTORs of the chosen offline clients are
dropped, which is how a late message looks to the server, :207-224).

Recorded (tests/golden/ref_golden.json + ref_golden.npz):
  * per client and iteration: m_i, the neighbour set in the reference's own
    iteration order, r_ij, h_ijt, s_ij, and the SHA-256 of the masked vector y_i;
  * per iteration on the server: arrival order, recon_symbol in order, the
    m_i / s_ij keys reconstruction_process actually fed to ChaCha20, and digests
    of vec_sum_partial, mi_vec (the no-dropout branch, :538-540, run on the same
    shares with a zero partial sum), cancel_vec and final_sum (the dropout
    branch, :541-605);
  * the decryptors' shares, the ElGamal c1 column and the Lagrange coefficients
    of the first iteration of variant A, so the GPU seed recovery can be run
    on the reference's own inputs;
  * findNeighbors / choose_committee outputs (util/param.py:38-103), including set
    iteration order, for N = 128 and 1024;
  * util/util.py:179-252 JSON strings of real messages (wire-format parity).

Reproduce:  python tests/golden/make_ref_golden.py   (~1-2 min, 8 cores)
"""
from __future__ import annotations

import contextlib
import copy
import hashlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
import refshim  # noqa: E402

refshim.install()
sys.path.insert(0, REF)
import pandas as pd  # noqa: E402
from util import param, util  # noqa: E402

util.read_key = refshim.read_key          # no PEM files: deterministic keys per file name
util.silent_mode = True
from util.crypto import ecchash  # noqa: E402
from util.crypto.secretsharing import points_to_secret_int  # noqa: E402
import agent.flamingo.SA_ClientAgent as CA  # noqa: E402
import agent.flamingo.SA_ServiceAgent as SA  # noqa: E402

ROOT = bytes(32)
param.root_seed = ROOT

H2C_LOG: list = []
_h2c = ecchash.hash_str_to_curve


def _h2c_logged(msg, count, modulus, degree, blen, expander):
    pt = _h2c(msg=msg, count=count, modulus=modulus, degree=degree, blen=blen, expander=expander)
    H2C_LOG.append((msg, int(pt.x), int(pt.y)))
    return pt


ecchash.hash_str_to_curve = _h2c_logged


def digest(v) -> str:
    return hashlib.sha256(np.ascontiguousarray(v, dtype="<u4").tobytes()).hexdigest()


def x_input(seed: int, it: int, cid: int, L: int) -> np.ndarray:
    """Random client input for the random-input variant (the reference uses all-ones, :304)."""
    return np.random.Generator(np.random.PCG64([seed, it, cid])).integers(0, 2**32, size=L, dtype=np.uint32)


class _NpProxy:
    """SA_ClientAgent's `np` with `ones` replaced by the current client's random input."""

    def __init__(self, seed):
        self.seed, self.cur = seed, None

    def __getattr__(self, k):
        return getattr(np, k)

    def ones(self, n, dtype=None):
        cid, it = self.cur
        return x_input(self.seed, it, cid, n).astype(dtype)


class StubKernel:
    def __init__(self, server_id):
        self.outbox, self.custom_state, self.server_id = [], {}, server_id

    def fmtTime(self, t):
        return t

    def sendMessage(self, sender, recipient, msg, delay=0, tag="communication"):
        self.outbox.append((sender, recipient, msg))

    def setWakeup(self, sender, requestedTime):
        pass

    def setAgentComputeDelay(self, sender, requestedDelay):
        pass

    def findAgentByType(self, t):
        return self.server_id

    def take(self, kind):
        out = [m for m in self.outbox if m[2].body["msg"] == kind]
        self.outbox = [m for m in self.outbox if m[2].body["msg"] != kind]
        return out


def run_protocol(name, N, L, o, offline_per_it, parallel_mode, x_seed=None, keep_recovery=False):
    """Drive len(offline_per_it) iterations through the reference agents; return (record, arrays)."""
    refshim.DRBG.reset(name.encode())
    param.vector_len = L
    proxy = None
    if x_seed is not None:
        proxy = _NpProxy(x_seed)
        CA.np = proxy
    else:
        CA.np = np
    iters = len(offline_per_it)
    kernel = StubKernel(N)
    clients = [CA.SA_ClientAgent(id=i, name=f"PPFL Client Agent {i}", type="ClientAgent", iterations=iters,
                                 num_clients=N, neighborhood_size=o, random_state=np.random.RandomState(i))
               for i in range(N)]
    server = SA.SA_ServiceAgent(id=N, name="PPFL Service Agent", type="ServiceAgent",
                                random_state=np.random.RandomState(N), msg_fwd_delay=0, users=[*range(N)],
                                iterations=iters, num_clients=N, neighborhood_size=o,
                                parallel_mode=parallel_mode)
    t = pd.Timestamp(0)
    for a in clients + [server]:
        a.kernel = kernel
        a.kernelStarting(t)                    # finds the service agent (SA_ClientAgent.py:119)
    refshim.TAG[0] = ("server", "initialize", 0)
    server.initialize(t)
    for _, rid, msg in kernel.take("COMMITTEE_SHARED_SK"):
        clients[rid].receiveMessage(t, msg)
    rec = {"name": name, "N": N, "L": L, "neighborhood_size": o, "parallel_mode": int(parallel_mode),
           "input": "ones (SA_ClientAgent.py:304)" if x_seed is None else
           f"x_input({x_seed}, it, i, L): PCG64([{x_seed}, it, i]).integers(0, 2**32, L, uint32)",
           "committee_order": [int(c) for c in server.user_committee], "iterations": []}
    arrays = {}
    arrival_rng = np.random.Generator(np.random.PCG64(len(name)))
    for it in range(1, iters + 1):
        del refshim.CHACHA_LOG[:]
        del H2C_LOG[:]
        clog = {}
        # --- clients: sendVectors (iteration 1 from wakeup, later ones from the REQ)
        pending_req = kernel.take("REQ")
        for c in clients:
            refshim.TAG[0] = ("client", c.id, it)
            if proxy is not None:
                proxy.cur = (c.id, it)
            n0 = len(H2C_LOG)
            if it == 1:
                c.wakeup(t)
            else:
                for _, rid, msg in pending_req:
                    if rid == c.id:
                        c.receiveMessage(t, msg)
            clog[c.id] = (list(c.neighbors_list), H2C_LOG[n0:])
        vec_msgs = kernel.take("VECTOR")
        assert len(vec_msgs) == N
        offline = sorted(offline_per_it[it - 1])
        order = [int(k) for k in arrival_rng.permutation(N)]
        by_sender = {m[2].body["sender"]: m for m in vec_msgs}
        clients_rec = []
        m_rows, seg, r_rows, s_rows, pts = [], [0], [], [], []
        for c in clients:
            keys = [(k, n) for tag, k, n in refshim.CHACHA_LOG if tag == ("client", c.id, it)]
            prg = [k for k, n in keys if n == 4 * L]
            hkeys = [k for k, n in keys if n == 16]
            nb, h2c = clog[c.id]
            assert len(prg) == 1 + len(nb) and len(hkeys) == len(nb) and len(h2c) == len(nb)
            body = by_sender[c.id][2].body
            clients_rec.append({"id": c.id, "neighbors": [int(j) for j in nb], "h": [h[0] for h in h2c],
                                "y_sha256": digest(body["vector"])})
            m_rows.append(prg[0])
            s_rows += prg[1:]
            r_rows += hkeys
            pts += [h[1].to_bytes(32, "big") + h[2].to_bytes(32, "big") for h in h2c]
            seg.append(len(s_rows))
        pre = f"{name}_it{it}_"
        arrays[pre + "m"] = np.frombuffer(b"".join(m_rows), np.uint8).reshape(-1, 32)
        arrays[pre + "pair_seg"] = np.array(seg, np.int64)
        arrays[pre + "r"] = np.frombuffer(b"".join(r_rows), np.uint8).reshape(-1, 32)
        arrays[pre + "s"] = np.frombuffer(b"".join(s_rows), np.uint8).reshape(-1, 32)
        arrays[pre + "h2c_point"] = np.frombuffer(b"".join(pts), np.uint8).reshape(-1, 64)
        for cid in order:
            if cid not in offline:
                refshim.TAG[0] = ("server", "recv", it)
                server.receiveMessage(t, by_sender[cid][2])
        refshim.TAG[0] = ("server", "report", it)
        with contextlib.redirect_stdout(io.StringIO()):
            server.report(t)
        S = server.vec_sum_partial.copy()
        recon = [[int(a), int(b), int(s)] for (a, b), s in server.recon_symbol.items()]
        arrival = [int(i) for i in server.client_id_list]
        # --- crosscheck + decryption shares
        for _, rid, msg in kernel.take("SIGN"):
            if rid == N:
                server.receiveMessage(t, msg)
            else:
                clients[rid].receiveMessage(t, msg)
        for _, rid, msg in kernel.take("SIGN"):          # the decryptors' signed labels
            server.receiveMessage(t, msg)
        with contextlib.redirect_stdout(io.StringIO()):
            server.forward_signatures(t)
        dec = kernel.take("DEC")
        for k in [int(v) for v in arrival_rng.permutation(len(dec))]:
            _, rid, msg = dec[k]
            clients[rid].receiveMessage(t, msg)
        shared = kernel.take("SHARED_RESULT")
        for _, rid, msg in shared:
            server.receiveMessage(t, msg)
        # --- reconstruction (the body of SA_ServiceAgent.reconstruction, :439-467)
        server.reconstruction_read_from_pool()
        snap = (copy.deepcopy(server.committee_shares_pairwise), copy.deepcopy(server.committee_shares_mi),
                dict(server.recon_index))
        threshold = server.committee_threshold
        dec_order = list(server.committee_shares_mi.keys())[:threshold]
        xs = [int(server.recon_index[d]) for d in dec_order]
        dec_c1 = [(int(v[1].x), int(v[1].y)) for v in server.dec_target_pairwise.values()]
        del refshim.CHACHA_LOG[:]
        refshim.TAG[0] = ("server", "recon", it)
        with contextlib.redirect_stdout(io.StringIO()):
            server.reconstruction_process()
        final = server.final_sum.copy()
        rkeys = [k for tag, k, n in refshim.CHACHA_LOG if tag == ("server", "recon", it) and n == 4 * L]
        M = len(arrival)
        assert len(rkeys) == M + len(recon)
        # the no-dropout branch (:538-540) on the same shares with a zero partial sum: final_sum = mi_vec
        dtp, symb = server.dec_target_pairwise, server.recon_symbol
        server.committee_shares_pairwise, server.committee_shares_mi, server.recon_index = copy.deepcopy(snap)
        server.vec_sum_partial = np.zeros(L, dtype=np.uint32)
        server.dec_target_pairwise = {}
        with contextlib.redirect_stdout(io.StringIO()):
            server.reconstruction_process()
        mi_vec = server.final_sum.copy()
        server.dec_target_pairwise, server.recon_symbol = dtp, symb
        server.final_sum = final
        server.reconstruction_clear_pool()
        server.reconstruction_send_message()
        server.current_round = 1
        server.current_iteration += 1
        cancel = (final - S - mi_vec).astype(np.uint32)
        arrays[pre + "server_m"] = np.frombuffer(b"".join(rkeys[:M]), np.uint8).reshape(-1, 32)
        arrays[pre + "server_pairs"] = np.frombuffer(b"".join(rkeys[M:]), np.uint8).reshape(-1, 32)
        online = sorted(set(range(N)) - set(offline))
        itrec = {"iteration": it, "offline": offline, "arrival": arrival, "recon_symbol": recon,
                 "S_sha256": digest(S), "M_sha256": digest(mi_vec), "C_sha256": digest(cancel),
                 "final_sha256": digest(final), "final_head": final[:8].tolist(),
                 "decryptor_order": [int(d) for d in dec_order], "decryptor_x": xs,
                 "clients": clients_rec}
        if x_seed is None:
            assert np.all(final == len(online)), "reference final_sum != |U| for all-ones inputs"
            itrec["final_value"] = len(online)
        else:
            want = np.zeros(L, np.uint32)
            for i in online:
                want += x_input(x_seed, it, i, L)
            assert np.array_equal(final, want), "reference final_sum != sum of online inputs"
        # Lagrange coefficients exactly as reconstruction_process gets them (:507-514)
        primary = [(server_x, 0) for server_x in xs]
        _, lam = points_to_secret_int(points=primary, prime=ecchash.n, isecc=0)
        itrec["lagrange"] = [hex(v) for v in lam]
        if keep_recovery and it == 1:
            shares_mi = np.zeros((threshold, M, 32), np.uint8)
            shares_pw = np.zeros((threshold, len(recon), 64), np.uint8)
            for tdx, d in enumerate(dec_order):
                for m, v in enumerate(snap[1][d]):
                    shares_mi[tdx, m] = np.frombuffer(int(v).to_bytes(32, "big"), np.uint8)
                for p, pt in enumerate(snap[0][d]):
                    shares_pw[tdx, p] = np.frombuffer(int(pt.x).to_bytes(32, "big") + int(pt.y).to_bytes(32, "big"),
                                                      np.uint8)
            arrays[f"{name}_it{it}_mi_shares"] = shares_mi
            arrays[f"{name}_it{it}_pair_shares"] = shares_pw
            arrays[f"{name}_it{it}_c1"] = np.array([np.frombuffer(x.to_bytes(32, "big") + y.to_bytes(32, "big"),
                                                                  np.uint8) for x, y in dec_c1], np.uint8
                                                   ).reshape(-1, 64)
            # util/util.py:179-252 strings of real messages (wire-format parity)
            vb = by_sender[arrival[0]][2].body
            itrec["wire"] = {
                "client": arrival[0],
                "enc_mi_shares": vb["enc_mi_shares"], "enc_pairwise": vb["enc_pairwise"],
                "shared_result_pairwise": shared[0][2].body["shared_result_pairwise"],
                "shared_result_mi": shared[0][2].body["shared_result_mi"],
                "dim2_ecp": util.serialize_dim2_ecp({str(d): snap[0][d][:3] for d in dec_order[:2]}),
            }
        rec["iterations"].append(itrec)
    CA.np = np
    return rec, arrays


def graphs():
    out = []
    for n, o, it in ((128, 1, 1), (128, 1, 2), (128, 2, 1), (1024, 1, 1), (1024, 2, 1)):
        nb = [list(param.findNeighbors(ROOT, it, n, i, o)) for i in range(n)]
        g = {"num_clients": n, "neighborhood_size": o, "iteration": it,
             "iter_order_sha256": hashlib.sha256(json.dumps(nb).encode()).hexdigest(),
             "sorted_sha256": hashlib.sha256(json.dumps([sorted(s) for s in nb]).encode()).hexdigest(),
             "degree_sum": sum(len(s) for s in nb)}
        if n == 128:
            g["neighbors"] = nb
        out.append(g)
    return out


def main():
    out = {"generator": "tests/golden/make_ref_golden.py: the reference's own util/param.py, util/util.py, "
                        "util/crypto and agent/flamingo/SA_{Client,Service}Agent.py imported read-only from "
                        "/root/reference under tests/golden/refshim.py",
           "root_seed": ROOT.hex(), "sqrtmod_assumption": "libnum.sqrtmod yields a^((p+1)/4) mod p first"}
    out["committee"] = [{"num_clients": n, "iter_order": [int(c) for c in param.choose_committee(ROOT, 60, n)]}
                        for n in (128, 1024, 4096)]
    out["graphs"] = graphs()
    print("graphs done", flush=True)
    arrays = {}
    runs = []
    for args in (dict(name="A", N=128, L=16384, o=1, offline_per_it=[[3, 77, 100], [13]], parallel_mode=1,
                      keep_recovery=True),
                 dict(name="B", N=128, L=16000, o=1, offline_per_it=[[10, 90]], parallel_mode=0, x_seed=20231015),
                 dict(name="C", N=128, L=16384, o=1, offline_per_it=[[]], parallel_mode=1),
                 # BASELINE c3's shape of graph: N = 1024 clients, neighbourhood -o 2 (config/flamingo.py:37-38),
                 # a few offline clients, so c3's pair ordering and recon_symbol are pinned directly
                 dict(name="D", N=1024, L=4096, o=2, offline_per_it=[[5, 300, 777, 1000]], parallel_mode=1)):
        rec, arr = run_protocol(**args)
        runs.append(rec)
        arrays.update(arr)
        print("run", args["name"], "done", flush=True)
    out["runs"] = runs
    with open(os.path.join(HERE, "ref_golden.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    np.savez_compressed(os.path.join(HERE, "ref_golden.npz"), **arrays)
    print("wrote ref_golden.json / ref_golden.npz")


if __name__ == "__main__":
    sys.exit(main())
