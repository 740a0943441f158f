"""Simulation-wide protocol state shared by the Flamingo agents (the role util/param.py plays).

Holds the root seed, the vector length and the committee parameters, the one
GPU engine of this process, and caches the committee and the per-iteration
neighbour graph (the reference re-derives the graph in every findNeighbors
call, util/param.py:56-103; here it is derived once per iteration for all
clients, with the keystream computed on the GPU).
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
_graphs: dict = {}
_committees: dict = {}
_pkis: dict = {}
_h2c: dict = {}


def configure(root: bytes | None = None, L: int | None = None, committee: int | None = None):
    """Reset the protocol parameters (between simulations / in tests)."""
    global root_seed, vector_len, committee_size
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


def engine():
    """The process's MaskEngine (created lazily: after any fork, before first use)."""
    global _engine
    if _engine is None:
        from ...engine import MaskEngine
        _engine = MaskEngine(int(os.environ.get("FLM_DEVICE", "0")))
    return _engine


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
    (SA_ClientAgent.py:283-286).  h_ijt is a decimal string below 2^16, so results are memoised."""
    pt = _h2c.get(h_ijt)
    if pt is None:
        from ...crypto import hash_str_to_curve
        pt = _h2c[h_ijt] = hash_str_to_curve(h_ijt)
    return pt
