"""Simulation-wide protocol state shared by the Flamingo agents (the role util/param.py plays).

Holds the root seed, the vector length and the committee parameters, the one
GPU engine of this process, and caches the committee and the per-iteration
neighbour graph (the reference re-derives the graph in every findNeighbors
call, util/param.py:56-103; here it is derived once per iteration for all
clients, with the keystream computed on the GPU).

The simulation's P-256 work is batched across clients, because one scalar
multiplication is a ~3 ms latency chain on the GPU whatever the batch size
(DESIGN.md section 5): every ECDH point a_i A_j of the iteration's graph and
of the client x committee pairs (symmetric, so one per unordered pair), and
every client's ElGamal r G, r pk of the iteration, are computed in one launch
each and handed to the agents.  The values are those each client would
compute alone (SA_ClientAgent.py:234-236, 256-263, 434-447).
"""
from __future__ import annotations

import os

from ... import params as P

root_seed: bytes = os.urandom(32)     # util/param.py:31 draws it at import time too
vector_len: int = P.vector_len       # util/param.py:8
vector_type = P.vector_type
committee_size: int = P.committee_size
fraction: float = P.fraction
nonce = P.nonce

_engine = None
_group = None
_graphs: dict = {}
_committees: dict = {}
_pkis: dict = {}
_h2c: dict = {}           # h_ijt -> point, memoised lookups of the GPU table
_h2c_table = None         # (out (65536, 64), flags): hash_str_to_curve(str(v)) for every v < 2^16
_ecdh: dict = {}          # (root, N, min(i,j), max(i,j)) -> 64-byte wire of a_i A_j
_ecdh_done: set = set()   # batches already computed (graph iterations, committee)
_clients: dict = {}       # id -> client agent (for the batched ElGamal draws)
_elgamal: dict = {}       # (root, iteration, id) -> (r list, (deg, 64) rG wire, (deg, 64) c1 = H + r pk wire)
_pair_keys: dict = {}     # (root, N, min(i,j), max(i,j)) -> r_ij = SHA-256(a_i A_j)[:32] (symmetric)
_pair_mat: dict = {}      # (root, iteration, N, nsize) -> {id: PairMaterial}


def configure(root: bytes | None = None, L: int | None = None, committee: int | None = None):
    """Reset the protocol parameters (between simulations / in tests)."""
    global root_seed, vector_len, committee_size, _h2c_table
    if root is not None:
        if len(root) != 32:
            raise ValueError("root seed must be 32 bytes")
        root_seed = root
    if L is not None:
        vector_len = int(L)
    if committee is not None:
        committee_size = int(committee)
    _graphs.clear()
    _committees.clear()
    _pkis.clear()
    _ecdh.clear()
    _ecdh_done.clear()
    _clients.clear()
    _elgamal.clear()
    _pair_keys.clear()
    _pair_mat.clear()
    _h2c.clear()                 # the table is the engine's: recomputed with whatever engine is current
    _h2c_table = None


def shutdown():
    """Close the server's device group (its RCCL clique included) and the process engine, after the
    stores on them are closed; the next engine()/server_engine() call starts afresh."""
    global _engine, _group
    configure()
    if _group is not None:
        _group.close()
        _group = None
    if _engine is not None:
        _engine.close()
        _engine = None


def engine():
    """The process's MaskEngine (created lazily: after any fork, before first use)."""
    global _engine
    if _engine is None:
        from ...engine import MaskEngine
        _engine = MaskEngine(int(os.environ.get("FLM_DEVICE", "0")))
    return _engine


def server_devices() -> list:
    """Devices the server's vector steps use: FLM_GROUP_DEVICES ("0,1,2,..."; one id repeated =
    loopback ranks on one GPU), else FLM_GPUS devices 0..n-1 (FLM_GPUS=all: every visible GPU),
    else the process's one device (FLM_DEVICE).  A multi-GPU group is opt-in."""
    spec = os.environ.get("FLM_GROUP_DEVICES", "").strip()
    if spec:
        return [int(d) for d in spec.split(",")]
    n = os.environ.get("FLM_GPUS", "").strip().lower()
    if n == "all":
        from ... import _lib
        return list(range(max(1, int(_lib.load().flm_device_count()))))
    if n and int(n) > 1:
        return list(range(int(n)))
    return [int(os.environ.get("FLM_DEVICE", "0"))]


def server_group_rccl() -> bool:
    """FLM_GROUP_RCCL=1: a one-device server group still gets an RCCL clique (flm_group_init_flags
    with FLM_GROUP_RCCL), so the drop-in server runs the multi-GPU code path on one GPU."""
    return os.environ.get("FLM_GROUP_RCCL", "").strip() not in ("", "0")


def server_engine():
    """The server's partial sum and unmask (SA_ServiceAgent.py:346-350, 529-605) run on every
    device of server_devices(): a DeviceGroup (client-sharded rows, slot-sharded masks, one RCCL
    reduce-scatter) when that is more than one (or FLM_GROUP_RCCL asks for a one-device clique),
    else the process MaskEngine.  Should the group not come up (RCCL missing, a device refused),
    the server says so and stays on one GPU.  The group is kept while the device list and the
    requested FLM_GROUP_RCCL flag stay the same (a group of distinct devices always has a clique,
    so it is the request that is compared, not flm_group_has_rccl).  A group replaced while a
    VectorStore still uses it is marked retired and closed by that store's close() (the agent swaps
    its store at the next iteration boundary, SA_ServiceAgent.reconstruction_clear_pool)."""
    global _group
    devs = server_devices()
    force = server_group_rccl()
    if len(devs) == 1 and devs[0] == int(os.environ.get("FLM_DEVICE", "0")) and not force:
        return engine()
    if _group is None or _group.devices != devs or _group.force_rccl != force:
        from ...engine import DeviceGroup
        if _group is not None:
            if _group._stores:
                _group.retired = True      # closed by its last VectorStore's close()
            else:
                _group.close()
            _group = None
        try:
            _group = DeviceGroup(devs, force_rccl=force)
        except RuntimeError as e:
            import warnings
            warnings.warn(f"server device group {devs} unavailable ({e}); using one GPU")
            return engine()
    return _group


def vector_store(L: int, capacity: int):
    """The server's device-resident VECTOR store (flamingo_amd.ingest.VectorStore) on
    server_engine()'s device(s).  An engine object that brings its own store (a test double)
    provides it through a `vector_store(L, capacity)` method."""
    eng = server_engine()
    own = getattr(eng, "vector_store", None)
    if own is not None:
        return own(L, capacity)
    from ...ingest import VectorStore
    return VectorStore(eng, L, capacity)


def committee(num_clients: int) -> set:
    key = (root_seed, committee_size, num_clients)
    if key not in _committees:
        _committees[key] = P.choose_committee(root_seed, committee_size, num_clients,
                                              encrypt=engine().chacha20_encrypt)
    return _committees[key]


def neighbors(iteration: int, num_clients: int, neighborhood_size: int) -> list:
    key = (root_seed, iteration, num_clients, neighborhood_size)
    if key not in _graphs:
        _graphs.clear() if len(_graphs) > 8 else None
        _graphs[key] = P.neighbor_graph(root_seed, iteration, num_clients, neighborhood_size,
                                        encrypt=engine().chacha20_encrypt)
    return _graphs[key]


def find_neighbors(root, current_iteration, num_clients, id, neighborhood_size) -> set:
    """util/param.findNeighbors signature."""
    if root != root_seed:
        return P.find_neighbors(root, current_iteration, num_clients, id, neighborhood_size,
                                encrypt=engine().chacha20_encrypt)
    return neighbors(current_iteration, num_clients, neighborhood_size)[id]


def pki(num_clients: int):
    """Key material for this simulation (pki_files/ stand-in, see pki.py)."""
    key = (root_seed, num_clients)
    if key not in _pkis:
        from .pki import PKI
        _pkis.clear()
        _pkis[key] = PKI(root_seed, num_clients, engine())
    return _pkis[key]


def hash_to_curve(h_ijt: str):
    """ecchash.hash_str_to_curve(h_ijt, 2, n, m, L, XMD-SHA256) as the client calls it
    (SA_ClientAgent.py:283-286), on the GPU.  h_ijt is str(x & 0xFFFF) (:280), so the first call
    computes the whole table of the 2^16 possible points in one launch
    (MaskEngine.hash_to_curve_decimal) and every later call is a lookup; any other message is
    hashed by its own launch.  Returns the affine point (x, y), or None for infinity."""
    pt = _h2c.get(h_ijt)
    if pt is not None:
        return pt
    if h_ijt.isdigit() and str(int(h_ijt)) == h_ijt and int(h_ijt) < (1 << 16):
        out, fl = h2c_table()
        row, f = out[int(h_ijt)], int(fl[int(h_ijt)])
    else:
        out, fl = engine().hash_to_curve_wire([h_ijt])
        row, f = out[0], int(fl[0])
    b = row.tobytes()
    pt = _h2c[h_ijt] = None if f & 4 else (int.from_bytes(b[:32], "big"), int.from_bytes(b[32:], "big"))
    return pt


# ------------------------------------------------------- batched P-256 work
def _ecdh_batch(num_clients: int, pairs) -> None:
    """a_i A_j for every (i, j) in pairs not cached yet, in one GPU launch.  i == j is kept: a
    committee member that is also a client encrypts its own m_i share under a_i A_i (:234-236)."""
    from ... import crypto as C
    import numpy as np
    kp = pki(num_clients)
    todo = sorted({(min(i, j), max(i, j)) for i, j in pairs} -
                  {k[2:] for k in _ecdh if k[:2] == (root_seed, num_clients)})
    if not todo:
        return
    a = [kp.client_sk[i] for i, _ in todo]
    out, _ = engine().ec_mul_wire(kp.pk_wire([j for _, j in todo]), C.scalars_to_wire(a))
    for (i, j), row in zip(todo, np.asarray(out)):
        _ecdh[(root_seed, num_clients, i, j)] = bytes(row)


def prefetch_graph_ecdh(iteration: int, num_clients: int, neighborhood_size: int) -> None:
    key = ("graph", root_seed, iteration, num_clients, neighborhood_size)
    if key in _ecdh_done:
        return
    nb = neighbors(iteration, num_clients, neighborhood_size)
    _ecdh_batch(num_clients, [(i, j) for i in range(num_clients) for j in nb[i]])
    _ecdh_done.add(key)


def prefetch_committee_ecdh(num_clients: int) -> None:
    key = ("committee", root_seed, num_clients, committee_size)
    if key in _ecdh_done:
        return
    comm = sorted(committee(num_clients))
    _ecdh_batch(num_clients, [(i, c) for i in range(num_clients) for c in comm])
    _ecdh_done.add(key)


def ecdh_wire(num_clients: int, i: int, j: int) -> bytes:
    """a_i A_j (= a_j A_i) as 64 wire bytes x||y; computed in a batch if not prefetched."""
    k = (root_seed, num_clients, min(i, j), max(i, j))
    if k not in _ecdh:
        _ecdh_batch(num_clients, [(i, j)])
    return _ecdh[k]


def h2c_table():
    """(out (65536, 64), flags) of hash_str_to_curve(str(v)) for every v < 2^16, one GPU launch
    (computed on first use, kept for the simulation)."""
    global _h2c_table
    if _h2c_table is None:
        _h2c_table = engine().hash_to_curve_decimal(0, 1 << 16)
    return _h2c_table


def pair_material(iteration: int, num_clients: int, neighborhood_size: int) -> dict:
    """Every client's pairwise seeds of `iteration` in a few batched launches
    (SA_ClientAgent.py:253-292): id -> (nb, h, H, s) with nb the neighbour list in the reference's
    set order, h the h_ijt strings, H the (deg, 64) wire rows of hash_str_to_curve(h_ijt) and s the
    32-byte seeds SHA-256(H).  r_ij = SHA-256(a_i A_j) comes from the graph's ECDH batch; every h_ijt
    of the iteration from ONE PRG launch (client_agent.pair_prf); H from the hash-to-curve table."""
    import hashlib
    import numpy as np
    key = (root_seed, iteration, num_clients, neighborhood_size)
    if key in _pair_mat:
        return _pair_mat[key]
    from .client_agent import pair_prf
    nbrs = neighbors(iteration, num_clients, neighborhood_size)
    prefetch_graph_ecdh(iteration, num_clients, neighborhood_size)
    lists = [list(nbrs[i]) for i in range(num_clients)]
    keys = []
    for i, nb in enumerate(lists):
        for j in nb:
            k = (root_seed, num_clients, min(i, j), max(i, j))
            r = _pair_keys.get(k)
            if r is None:
                r = _pair_keys[k] = hashlib.sha256(ecdh_wire(num_clients, i, j)).digest()[:32]
            keys.append(r)
    hs = pair_prf(engine(), keys, iteration)
    out, fl = h2c_table()
    rows = [np.asarray(out[int(h)], np.uint8) for h in hs]
    mat, o = {}, 0
    for i, nb in enumerate(lists):
        n = len(nb)
        H = np.stack(rows[o:o + n]) if n else np.zeros((0, 64), np.uint8)
        if n and any(int(fl[int(h)]) & 4 for h in hs[o:o + n]):
            raise RuntimeError("hash_to_curve gave the point at infinity")      # not in the 2^16 table
        mat[i] = (nb, hs[o:o + n], H, [hashlib.sha256(r.tobytes()).digest() for r in H])
        o += n
    for k in [k for k in _pair_mat if k[1] < iteration - 1]:
        del _pair_mat[k]
    _pair_mat[key] = mat
    return mat


def register_client(agent) -> None:
    _clients[agent.id] = agent


def elgamal_masks(agent, iteration: int, nb: list):
    """(r list, c0 = r G wire rows, c1 = H + r pk_system wire rows) for this client's neighbours in
    `iteration` (SA_ClientAgent.py:326-332, 434-447), H the pair's hash-to-curve point
    (pair_material).  The first client to ask in an iteration draws every registered, online
    client's r's from that client's own random state and computes all of them in two launches:
    r G and r pk (flm_ec_mul), then H + r pk (flm_ec_combine with one term of coefficient 1)."""
    from ... import crypto as C
    import numpy as np
    key = (root_seed, iteration, agent.id)
    if key not in _elgamal:
        batch = []
        for cid in sorted(_clients):
            c = _clients[cid]
            if iteration in c.offline_iterations or (root_seed, iteration, cid) in _elgamal:
                continue
            cnb = list(neighbors(iteration, c.num_clients, c.neighborhood_size)[cid])
            batch.append((cid, [c._rand_scalar() for _ in cnb]))
        if agent.id not in [b[0] for b in batch]:
            batch.append((agent.id, [agent._rand_scalar() for _ in nb]))
        rs = [r for _, r_list in batch for r in r_list]
        if rs:
            sys_pk = pki(agent.num_clients).system_pk
            base = np.concatenate([np.tile(np.frombuffer(C.point_bytes(C.G), np.uint8), (len(rs), 1)),
                                   np.tile(np.frombuffer(C.point_bytes(sys_pk), np.uint8), (len(rs), 1))])
            out, _ = engine().ec_mul_wire(base, C.scalars_to_wire(rs + rs))
            out = np.asarray(out)
            pm = pair_material(iteration, agent.num_clients, agent.neighborhood_size)
            H = np.concatenate([pm[cid][2] for cid, r_list in batch if r_list])
            c1, _, fl = engine().ec_combine_wire(H, out[len(rs):][None], C.scalars_to_wire([1]), negate=False)
            c1 = np.asarray(c1)
            if (np.asarray(fl) & 4).any():
                raise RuntimeError("ElGamal c1 = H + r pk at infinity")
        o = 0
        for cid, r_list in batch:
            n = len(r_list)
            _elgamal[(root_seed, iteration, cid)] = (r_list, out[o:o + n] if n else None, c1[o:o + n] if n else None)
            o += n
        for k in [k for k in _elgamal if k[1] < iteration - 1]:
            del _elgamal[k]
    return _elgamal.pop(key)
