"""Sharded (multi-GPU) hash stage: the exchange protocol of sharded.py on CPU.

world_size 2 and 4 over gloo, each rank a numpy model of the per-rank compute
(tests/dist_model.py).  Concatenating the ranks' dispatch in descending rank
order must give the oracle's single-process wide-id dispatch and counts
exactly; the role pairs summed over the owners must equal the oracle's.
The HIP worker runs the same orchestration in tests/test_gpu_parity.py.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import helpers as H


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, P, port, reads, starts, settings, outdir, budget=None):
    import torch.distributed as dist

    from dist_model import NumpyWorker
    from sharded import ShardedOverlapper

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        lengths = [len(r) for r in reads]
        w = NumpyWorker(reads[starts[rank]:starts[rank + 1]], **settings)
        so = ShardedOverlapper(w, rank, P, starts, lengths, "cpu")
        so.build(budget)
        so.build(budget)  # a second step reuses the exchange buffers
        np.savez(os.path.join(outdir, "r%d.npz" % rank), lead=w.lead, trail=w.trail, count=w.dcount,
                 rp=np.int64(w.role_pairs), xb=np.int64(so.exchanged_bytes), npass=np.int64(so.npass))
    finally:
        dist.destroy_process_group()


def run_sharded(reads, starts, settings, tmp_path, budget=None, npass_out=None):
    P = len(starts) - 1
    mp.spawn(_rank_main, args=(P, free_port(), reads, list(starts), settings, str(tmp_path), budget), nprocs=P)
    res = [np.load(os.path.join(str(tmp_path), "r%d.npz" % r)) for r in range(P)]
    order = list(range(P - 1, -1, -1))  # leads descend across ranks
    lead = np.concatenate([res[r]["lead"] for r in order])
    trail = np.concatenate([res[r]["trail"] for r in order])
    count = np.concatenate([res[r]["count"] for r in order])
    if npass_out is not None:
        npass_out.extend(int(x["npass"]) for x in res)
    return lead, trail, count, int(sum(int(x["rp"]) for x in res)), [int(x["xb"]) for x in res]


def oracle_dispatch_counts(r):
    key = {(int(a), int(b)): int(c) for a, b, c in zip(r.pair_fst, r.pair_snd, r.pair_cnt)}
    return np.array([key[(int(a), int(b))] for a, b in zip(r.lead, r.trail)], dtype=np.int32)


@pytest.mark.parametrize("P", [2, 4])
def test_sharded_protocol_matches_oracle(oracle_mod, P, tmp_path):
    reads = H.synth_reads(240, 120, 2400, gc=0.5, seed=61 + P, mixed=(60, 160))
    # uneven shards (the last one largest), one rank may hold few reads
    cut = sorted({0, len(reads)} | {int(len(reads) * f) for f in np.linspace(0.15, 0.7, P - 1)})
    assert len(cut) == P + 1
    settings = dict(k=12, min_c=3, max_c=222)
    lead, trail, count, rp, xb = run_sharded(reads, cut, settings, tmp_path)
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(kmer_size=12, min_collisions=3),
                       wide=True, skip_align=True)
    assert len(r.lead) > 200
    np.testing.assert_array_equal(lead, r.lead)
    np.testing.assert_array_equal(trail, r.trail)
    np.testing.assert_array_equal(count, oracle_dispatch_counts(r))
    assert all(x > 0 for x in xb)  # every rank sent records to its peers


def test_sharded_single_rank_is_the_whole_job(oracle_mod, tmp_path):
    reads = H.synth_reads(90, 100, 900, seed=67)
    lead, trail, count, rp, xb = run_sharded(reads, [0, len(reads)], dict(k=11, min_c=2), tmp_path)
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(kmer_size=11, min_collisions=2),
                       wide=True, skip_align=True)
    np.testing.assert_array_equal(lead, r.lead)
    np.testing.assert_array_equal(trail, r.trail)
    assert xb == [0]


@pytest.mark.parametrize("P,budget", [(2, 3000), (4, 1500), (4, 10 ** 9)])
def test_sharded_lead_range_passes_match_oracle(oracle_mod, P, budget, tmp_path):
    """The count in lead-range passes (sa_dist_buckets / _plan / _count_pass /
    _reduce_pass protocol): every rank plans its passes within `budget` partial
    entries, the ranks run the largest plan, and per pass only the leads of each
    owner's slice are counted, exchanged and reduced -- the dispatch is the
    single-pass one (the oracle's), pass after pass appended lead-descending."""
    reads = H.synth_reads(240, 120, 2400, gc=0.5, seed=81 + P, mixed=(60, 160))
    cut = [len(reads) * r // P for r in range(P + 1)]
    npass = []
    lead, trail, count, rp, xb = run_sharded(reads, cut, dict(k=12, min_c=3, max_c=222), tmp_path, budget, npass)
    r = oracle_mod.Run(reads=reads, settings=oracle_mod.default_settings(kmer_size=12, min_collisions=3),
                       wide=True, skip_align=True)
    np.testing.assert_array_equal(lead, r.lead)
    np.testing.assert_array_equal(trail, r.trail)
    np.testing.assert_array_equal(count, oracle_dispatch_counts(r))
    assert len(set(npass)) == 1  # one plan for every rank
    assert (npass[0] > 1) == (budget < 10 ** 9)
