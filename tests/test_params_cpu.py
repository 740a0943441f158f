"""CPU checks of the product-side host round logic (flamingo_amd/params.py) against the per-id
oracle restatement of util/param.py and the committed OpenSSL fixtures.  The product functions
take their ChaCha20 keystream as a parameter (the GPU engine in production); here the oracle's
keystream stands in, as test infrastructure, so only the host logic is under test."""
import hashlib
import json

import numpy as np
import pytest

import oracle as O
from flamingo_amd import params as P

ROOT0 = bytes(32)


@pytest.mark.parametrize("n,o,it", [(128, 1, 1), (128, 1, 2), (1024, 1, 1), (1024, 2, 1)])
def test_neighbor_graph_matches_fixtures(golden, n, o, it):
    """All-clients-at-once graph == the reference's per-call findNeighbors (util/param.py:56-103)."""
    e = next(g for g in golden["graphs"] if (g["num_clients"], g["neighborhood_size"], g["iteration"]) == (n, o, it))
    nb = P.neighbor_graph(ROOT0, it, n, o, encrypt=O.chacha20_encrypt)
    assert [sorted(nb[i]) for i in range(8)] == e["first8"]
    if n <= 128:
        assert hashlib.sha256(json.dumps([sorted(x) for x in nb]).encode()).hexdigest() == e["sha256"]
    else:
        for i in (0, 1, 511, n - 1):
            assert nb[i] == O.find_neighbors(ROOT0, it, n, i, o)
    # symmetric, no self loops (SA_ClientAgent.py:323-324 guard)
    assert all(i not in nb[i] and all(i in nb[j] for j in nb[i]) for i in range(n))


def test_committee_matches_fixtures(golden):
    for e in golden["committee"]:
        assert sorted(P.choose_committee(ROOT0, 60, e["num_clients"], encrypt=O.chacha20_encrypt)) == e["members"]


def test_find_neighbors_drop_in():
    assert P.find_neighbors(ROOT0, 3, 256, 17, 1, encrypt=O.chacha20_encrypt) == \
        O.find_neighbors(ROOT0, 3, 256, 17, 1)


def test_dropout_pairs_and_server_table(round128):
    """(online nb, offline id) pairs with recon_symbol (SA_ServiceAgent.py:359-380) and the server seed
    table: -1 for every online m_i, then sigma for each pair, in the same pair order."""
    r = round128
    N = 128
    nb = P.neighbor_graph(ROOT0, 1, N, 1, encrypt=O.chacha20_encrypt)
    online = r["online"]
    offline = np.setdiff1d(np.arange(N), online)
    pairs, signs = P.dropout_pairs(nb, online, offline)
    want_pairs, want_signs = O.dropout_pairs(ROOT0, 1, N, 1, set(online.tolist()))
    assert sorted(zip(pairs, signs)) == sorted(zip(want_pairs, want_signs))
    assert sorted(pairs) == sorted(map(tuple, r["pairs"].tolist()))
    assert all(s == (1 if i > j else -1) for (i, j), s in zip(pairs, signs))
    m = np.arange(N * 32, dtype=np.uint32).astype(np.uint8).reshape(N, 32)
    seeds, sg = P.server_seed_table(m, nb, online, offline, P.synthetic_pair_seed)
    nU = len(online)
    assert seeds.shape == (nU + len(pairs), 32) and np.all(sg[:nU] == -1)
    assert np.array_equal(seeds[:nU], m[online])
    assert [bytes(s) for s in seeds[nU:]] == [P.synthetic_pair_seed(i, j) for i, j in pairs]
    assert sg[nU:].tolist() == signs


def test_client_seed_table_layout():
    """CSR rows: m_i with +1, then s_ij for j in N(i) with +1 if i < j else -1 (SA_ClientAgent.py:304-324)."""
    nb = [{1, 3}, {0}, set(), {0}]
    m = np.arange(4 * 32, dtype=np.uint8).reshape(4, 32)
    seg, seeds, signs = P.client_seed_table(m, nb, P.synthetic_pair_seed)
    assert seg.tolist() == [0, 3, 5, 6, 8]
    assert signs.tolist() == [1, 1, 1, 1, -1, 1, 1, -1]
    assert bytes(seeds[1]) == P.synthetic_pair_seed(0, 1) == P.synthetic_pair_seed(1, 0)
    with pytest.raises(RuntimeError):
        P.client_seed_table(m[:1], [{0}], P.synthetic_pair_seed)
