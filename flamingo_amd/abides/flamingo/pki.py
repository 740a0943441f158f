"""Key material of a simulated Flamingo deployment (the role of pki_files/).

The reference generates random P-256 keys once (pki_files/setup_pki.py) and
every agent reads PEM files: client{i}.pem (client key pair, used for ECDH
with neighbours and committee members, SA_ClientAgent.py:59-63) and
system_pk.pem (the decryption key the committee shares, :57,
SA_ServiceAgent.py:262-265).  Here the private keys are derived from the
simulation's root seed (reproducible runs, nothing on disk) and the public
keys are computed in one GPU batch (flm_ec_mul) for all clients.
"""
from __future__ import annotations

import hashlib

import numpy as np

from ... import crypto as C


def _derive(root: bytes, label: bytes) -> int:
    return int.from_bytes(hashlib.sha512(b"flm-pki" + root + label).digest(), "big") % (C.N - 1) + 1


class PKI:
    def __init__(self, root: bytes, num_clients: int, engine):
        self.num_clients = num_clients
        self.client_sk = [_derive(root, b"client%d" % i) for i in range(num_clients)]
        self.system_sk = _derive(root, b"system")
        self.server_sk = _derive(root, b"server")       # pki_files/server_key.pem (signs the offline set)
        sks = self.client_sk + [self.system_sk, self.server_sk]
        gw = np.tile(np.frombuffer(C.point_bytes(C.G), np.uint8), (len(sks), 1))
        out, _ = engine.ec_mul_wire(gw, C.scalars_to_wire(sks))
        pts = C.points_from_wire(out)
        self.client_pk = pts[:num_clients]
        self.system_pk = pts[num_clients]
        self.server_pk = pts[num_clients + 1]
        self._pk_wire = out[:num_clients]

    def pk_wire(self, ids) -> np.ndarray:
        """(len(ids), 64) wire rows of the clients' public keys (for batched ECDH)."""
        return self._pk_wire[np.asarray(list(ids), dtype=np.int64)]
