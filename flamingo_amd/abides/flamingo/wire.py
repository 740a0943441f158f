"""Message payload formats of the Flamingo agents (util/util.py:179-252).

The reference ships EC points and ciphertexts between agents as JSON strings;
these functions produce and parse the same JSON.  Points are (x, y) integer
tuples here (pycryptodome's EccPoint is not available); the JSON is the same
because the reference serialises int(p.x), int(p.y).

For the GPU, ``*_to_wire`` variants parse straight into (n, 64) uint8 arrays
of big-endian x||y (flamingo_hip.h's point format) without building Python
point objects.
"""
from __future__ import annotations

import json

import numpy as np


def serialize_dim1_elgamal(elgamal_dict) -> str:
    """{(i, j): (c0, c1)} -> '{"[i, j]": [c0x, c0y, c1x, c1y]}' (util.py:221-228)."""
    # f"[{i}, {j}]" is json.dumps([i, j]) for int ids, without a dumps call per key
    return json.dumps({f"[{int(k[0])}, {int(k[1])}]": (int(c0[0]), int(c0[1]), int(c1[0]), int(c1[1]))
                       for k, (c0, c1) in elgamal_dict.items()})


def deserialize_dim1_elgamal(s: str) -> dict:
    return {tuple(json.loads(k)): ((v[0], v[1]), (v[2], v[3])) for k, v in json.loads(s).items()}


def serialize_dim1_ecp(points) -> str:
    """[P0, P1, ...] -> '{"0": [x, y], ...}' (util.py:203-210)."""
    return json.dumps({i: (int(p[0]), int(p[1])) for i, p in enumerate(points)})


def deserialize_dim1_ecp(s: str) -> list:
    return [(v[0], v[1]) for v in json.loads(s).values()]


def serialize_dim2_ecp(ecp_dict) -> str:
    """{i: [P, ...]} -> '{"i": {"0": [x, y], ...}}' (util.py:179-188)."""
    return json.dumps({i: {j: (int(p[0]), int(p[1])) for j, p in enumerate(v)} for i, v in ecp_dict.items()})


def deserialize_dim2_ecp(s: str) -> dict:
    return {i: [(p[0], p[1]) for p in v.values()] for i, v in json.loads(s).items()}


def serialize_tuples_bytes(items) -> str:
    """[(ct, nonce), ...] -> '[["hex", "hex"], ...]' (util.py:239-242)."""
    # the json.dumps text of [[hex, hex], ...], built directly (hex digits need no escaping)
    return "[" + ", ".join(f'["{a.hex()}", "{b.hex()}"]' for a, b in items) + "]"


def deserialize_tuples_bytes(s: str) -> list:
    return [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in json.loads(s)]


def serialize_dim1_list(ls) -> str:
    return json.dumps(ls)


def deserialize_dim1_list(s: str) -> list:
    return json.loads(s)


# ------------------------------------------------------------ GPU batches
def _ints_to_wire(vals) -> np.ndarray:
    """Flat sequence of coordinate ints -> (n/2, 64) uint8 big-endian rows."""
    b = b"".join(int(v).to_bytes(32, "big") for v in vals)
    return np.frombuffer(b, np.uint8).reshape(-1, 64).copy()


def elgamal_json_to_wire(s: str):
    """serialize_dim1_elgamal JSON -> (keys, c0 (D,64), c1 (D,64))."""
    d = json.loads(s)
    keys = [tuple(json.loads(k)) for k in d]
    if not keys:
        return keys, np.zeros((0, 64), np.uint8), np.zeros((0, 64), np.uint8)
    c0 = _ints_to_wire(v for vals in d.values() for v in vals[:2])
    c1 = _ints_to_wire(v for vals in d.values() for v in vals[2:])
    return keys, c0, c1


def ecp_json_to_wire(s: str) -> np.ndarray:
    """serialize_dim1_ecp JSON -> (n, 64)."""
    d = json.loads(s)
    if not d:
        return np.zeros((0, 64), np.uint8)
    return _ints_to_wire(v for p in d.values() for v in p)


def wire_to_ecp_json(w: np.ndarray) -> str:
    """(n, 64) wire rows -> serialize_dim1_ecp JSON."""
    return json.dumps({i: (int.from_bytes(bytes(r[:32]), "big"), int.from_bytes(bytes(r[32:]), "big"))
                       for i, r in enumerate(w)})
