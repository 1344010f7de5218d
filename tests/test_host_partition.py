"""sheep_partition (the product's host forwardPartition, partition.cpp:50-157, through the C-ABI;
no GPU call) against the reference's published hep-th results and the checker."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def test_partition_hep_th_published_and_checker(oracle, hep_edges):
    from sheep_amd import api

    pub = json.load(open(os.path.join(GOLDEN, "hep_th_published.json")))
    seq = oracle.degree_sequence(hep_edges)
    parent, pst = oracle.build_tree(hep_edges, seq)
    ks = list(range(2, 33))  # one partition_tree run over every k (scripts/part-worker.sh:24)
    parts, created = api.partition(api.JNodeTable(parent, pst), seq, ks)
    ref = oracle.PartTree(parent, pst)
    for k, p, c in zip(ks, parts, created):
        assert np.array_equal(p, ref.partition(seq, k)), k
        rec = next(r for r in pub["partitions"] if r["k"] == k)
        assert c == rec["created"]
        assert (int((p == 0).sum()), int((p == 1).sum())) == (rec["size0"], rec["size1"])
        assert oracle.evaluate(hep_edges, p, seq)["ecv_down"] == rec["ecv_down"]


def test_partition_rejects_bad_arguments():
    from sheep_amd import api, capi

    t = api.JNodeTable(np.array([1, capi.INVALID], np.uint32), np.array([1, 1], np.uint32))
    seq = np.array([5, 3], np.uint32)
    parts, created = api.partition(t, seq, [1, 2])
    assert parts[0].size == 6 and parts[0][4] == -1 and created == [1, 2]
    assert (parts[1][5], parts[1][3]) == (0, 1)
    with pytest.raises(capi.SheepError):
        api.partition(t, seq, [0])
    with pytest.raises(capi.SheepError):  # a vertex heavier than total/k: refused, no hang
        api.partition(api.JNodeTable(t.parent, np.array([5, 0], np.uint32)), seq, [2])
