"""bench.py -- MI355X hash-overlap stage benchmark (BASELINE.json configs[1] and [2]).

Workload: a synthetic splitmix64 genome of
2.5 Mbp per GPU (GC 0.50, seed 1), 100,000 error-free forward reads of 500 bp
per GPU (20x coverage), k = 15, reference defaults otherwise, wide ids
(N >= 32,768 is outside the reference's 16-bit id domain).

A step = one pass of the hash stage over the device-resident reads:
pack -> k-mer emit -> (hash, loc) radix sort -> bucket/list build ->
edge<->middle pair count + collision filter -> candidate ordering
(KmerTable.calcPairData + calcDispatchData).  `value` = candidate k-mer (role)
pairs per second summed over ranks.  The end-to-end config (banded HOXD
dovetail alignment of every dispatched pair) is timed in a second loop and
reported as aligned_read_pairs_per_s.

Multi-GPU: one process per GPU (torchrun), backend "nccl"
(RCCL over xGMI).  Weak scaling: the genome grows with the GPU count (20x
coverage kept), each rank holds 100,000 reads of it (global ids by rank), and
a step is the SHARDED hash stage -- local k-mer emit, all-to-all of the
records to the rank owning their hash range, bucket build + partial pair
counts there, all-to-all of the partials to the rank owning the lead,
reduce + collision filter (sharded.py).  Reads are all-gathered once for the
alignment of each rank's own leads.  Barrier + max-over-ranks timing;
`value` sums the role pairs over all ranks.  `--replicas` runs independent
per-rank datasets instead (no exchange), for comparison.
"""
import argparse
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sequence-aligner_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec


def splitmix64(seed, n):
    """n consecutive outputs of splitmix64 starting from `seed` (vectorised)."""
    x = (np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
    z = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_lengths(n_reads, read_len, min_len, seed, shard=0):
    """Read lengths: all read_len, or U[min_len, read_len] from splitmix64 (BASELINE
    configs[4]'s mixed 100-1000 bp reads)."""
    if min_len is None or min_len >= read_len:
        return np.full(n_reads, read_len, dtype=np.int64)
    with np.errstate(over="ignore"):
        z = splitmix64((seed ^ 0x5EED) + 104729 * shard, n_reads)
    return (min_len + (z % np.uint64(read_len - min_len + 1))).astype(np.int64)


def synth_workload(n_reads, read_len, genome_len, gc, seed, shard=0, min_len=None):
    """Genome: base i from splitmix64(seed) (GC with probability gc); reads start
    uniformly in [0, G-L] (splitmix64((seed ^ 0xABCDEF) + 7919 * shard): shard
    r of a multi-GPU run samples its own reads of the same genome), forward
    strand, error-free; lengths from synth_lengths."""
    lens = synth_lengths(n_reads, read_len, min_len, seed, shard)
    with np.errstate(over="ignore"):
        z = splitmix64(seed, genome_len)
        u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
        bit = (z & np.uint64(1)).astype(np.uint8)
        genome = np.where(u < gc, np.where(bit == 1, ord("G"), ord("C")),
                          np.where(bit == 1, ord("T"), ord("A"))).astype(np.uint8)
        rs = (seed ^ 0xABCDEF) + 7919 * shard
        starts = (splitmix64(rs, n_reads) % (np.uint64(genome_len + 1) - lens.astype(np.uint64))).astype(np.int64)
    offsets = np.zeros(n_reads + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum(lens)
    if lens.min() == lens.max():
        idx = starts[:, None] + np.arange(read_len, dtype=np.int64)[None, :]
        return genome[idx].reshape(-1), offsets
    read_of = np.repeat(np.arange(n_reads, dtype=np.int64), lens)
    pos = np.arange(int(offsets[-1]), dtype=np.int64) - offsets[:-1].astype(np.int64)[read_of]
    return genome[starts[read_of] + pos], offsets


def pmc_traffic(kernels):
    """HBM bytes per step of the named kernels (substrings) from the newest
    committed PMC summary (profiles/*/pmc_summary_*.csv, written from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench by
    tools_profile.sh): sum of (FETCH_SIZE + WRITE_SIZE) KiB x 1024 per
    dispatch, uncorrected."""
    import csv
    import glob
    def natural(path):  # pmc_summary_v9 < pmc_summary_v10
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", path)]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary_*.csv")), key=natural)
    for path in reversed(files):
        with open(path) as f:
            rows = list(csv.DictReader(f))
        tot, found = 0.0, 0
        for kname in kernels:
            for row in rows:
                if kname in row["kernel"] and row.get("FETCH_SIZE_avg") and row.get("WRITE_SIZE_avg"):
                    tot += (float(row["FETCH_SIZE_avg"]) + float(row["WRITE_SIZE_avg"])) * 1024.0
                    found += 1
                    break
        if found == len(kernels):
            return int(tot), os.path.relpath(path, ROOT)
    return None, None


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=100_000)
    ap.add_argument("--len", type=int, default=500)
    ap.add_argument("--min-len", type=int, default=None,
                    help="mixed lengths U[min-len, len] (configs[4]: 100..1000); default: all --len")
    ap.add_argument("--k", type=int, default=15)
    ap.add_argument("--gc", type=float, default=0.50)
    ap.add_argument("--coverage", type=float, default=20.0)
    ap.add_argument("--align-steps", type=int, default=None)
    ap.add_argument("--cpu-sample-reads", type=int, default=100_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--quadratic-steps", type=int, default=0,
                    help="also time --quadratic-align (full-matrix local alignment) over the same dispatch")
    ap.add_argument("--align-kernel", type=int, default=0,
                    help="SA_OPT_ALIGN_KERNEL: 0 auto, 1 lane-group (LDS), 2 lane-per-pair")
    ap.add_argument("--replicas", action="store_true", help="N>1: independent per-rank datasets, no exchange")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) or gloo (host-staged, testing)")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    dist = None
    sharded = ws > 1 and not args.replicas
    if ws > 1:
        import torch
        import torch.distributed as dist_
        dist = dist_
        ndev = torch.cuda.device_count()
        local = local % max(ndev, 1)  # (gloo tests may run several ranks on one GPU)
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)

    import saoverlap as sao

    mean_len = args.len if args.min_len is None else (args.len + args.min_len) / 2.0
    G = int(args.reads * mean_len / args.coverage)
    if sharded:
        # one genome for all ranks (G per GPU, weak scaling), rank r's reads are
        # global ids r*reads+1 .. (r+1)*reads
        bases, offsets = synth_workload(args.reads, args.len, G * ws, args.gc, seed=1, shard=rank,
                                        min_len=args.min_len)
    else:
        bases, offsets = synth_workload(args.reads, args.len, G, args.gc, seed=1 + rank, min_len=args.min_len)
    ov = sao.Overlapper(device=local if ws > 1 else 0, timing=True, kmer_size=args.k,
                        id_mode=sao.SA_IDS_WIDE, align_kernel=args.align_kernel)
    ov.add_packed(bases.tobytes(), offsets)
    so = None
    if sharded:
        from sharded import HipWorker, ShardedOverlapper
        starts = np.arange(ws + 1, dtype=np.int64) * args.reads
        lengths = np.concatenate([synth_lengths(args.reads, args.len, args.min_len, 1, r)
                                  for r in range(ws)]).astype(np.int32)
        so = ShardedOverlapper(HipWorker(ov), rank, ws, starts, lengths, "cuda:%d" % local)
    build_step = so.build if so is not None else ov.device_build
    red_dev = "cuda" if args.dist_backend == "nccl" else "cpu"

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    # ---- hash stage (configs[1]) ------------------------------------------
    build_step()  # allocations happen here, outside the timed region
    for _ in range(args.warmup):
        build_step()
    ov.reset_stage_times()
    xb0 = so.exchanged_bytes if so is not None else 0
    barrier()
    ov.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        build_step()
    ov.sync()
    barrier()
    t_build = max_over_ranks(time.perf_counter() - t0)
    st = ov.stats()
    stages = ov.stage_times()
    role_pairs_total = sum_over_ranks(float(st["role_pairs"])) * args.steps
    value = role_pairs_total / t_build

    # ---- end-to-end incl. banded HOXD alignment (configs[2]) --------------
    asteps = args.align_steps if args.align_steps is not None else max(1, args.steps // 2)
    xbytes = (so.exchanged_bytes - xb0) / max(args.steps, 1) if so is not None else 0
    t_gather = None
    if so is not None:  # the reads every rank needs to align its own leads
        barrier()
        t0 = time.perf_counter()
        so.gather_reads()
        ov.sync()
        barrier()
        t_gather = max_over_ranks(time.perf_counter() - t0)
    ov.device_align()
    ov.reset_stage_times()
    barrier()
    ov.sync()
    t0 = time.perf_counter()
    for _ in range(asteps):
        ov.device_align()
    ov.sync()
    barrier()
    t_align = max_over_ranks(time.perf_counter() - t0)
    ast = ov.stats()
    astages = ov.stage_times()
    aligned_total = sum_over_ranks(float(ast["aligned"])) * asteps

    # ---- --quadratic-align (generateLocalAlignmentSet) over the same dispatch
    quad = None
    if args.quadratic_steps > 0:
        ov.set_aligner(sao.SA_ALIGNER_QUADRATIC)
        ov.device_align()  # allocation + warm-up
        ov.reset_stage_times()
        barrier()
        ov.sync()
        t0 = time.perf_counter()
        for _ in range(args.quadratic_steps):
            ov.device_align()
        ov.sync()
        barrier()
        t_quad = max_over_ranks(time.perf_counter() - t0)
        qst = ov.stats()
        quad = {"aligned_read_pairs_per_s": round(sum_over_ranks(float(qst["aligned"])) * args.quadratic_steps
                                                  / t_quad, 1),
                "ms_per_step": round(t_quad / args.quadratic_steps * 1e3, 3),
                "dp_cells_per_step": int(qst["dp_cells"]),
                "gcups": round(sum_over_ranks(float(qst["dp_cells"])) * args.quadratic_steps / t_quad / 1e9, 1)}
        ov.set_aligner(sao.SA_ALIGNER_LINEAR)

    # ---- roofline of the dominant hash-stage kernel ----------------------
    # By time the bucket build dominates the step: part_bounds + part_build<1024>
    # + part_build<2048> + part_build<4096> (the "buckets" stage, one HIP-event scope).  Algorithmic
    # HBM bytes per step: per k-mer 8 B (record load) + 16 B
    # (partner record store), + 4 B per partner-list entry (st/md/en tags of
    # every position: E2 cut table for each read length).  The partition starts
    # are binary searches (np log2 n cached loads), not a pass over the records.
    f32 = np.float32
    edge, center = f32(0.4), f32(0.4)
    lens_here = np.diff(offsets.astype(np.int64))
    list_entries = 0.0
    for L, nL in zip(*np.unique(lens_here, return_counts=True)):
        d = int(L) - args.k
        if d <= 0:
            continue
        loc = np.arange(d + 1, dtype=np.float32) / np.float32(d)
        tags = ((loc <= edge).astype(np.int64) + ((f32(0.5) - center * f32(0.5) <= loc) &
                (loc <= f32(0.5) + center * f32(0.5))).astype(np.int64) + (f32(1.0) - edge <= loc).astype(np.int64))
        list_entries += float(nL) * float(tags.sum())
    if sharded:  # this rank builds the buckets it owns: ~1/ws of all k-mers
        list_entries *= st["kmers"] / max(1.0, float(np.sum(np.maximum(lens_here - args.k + 1, 0))))
    bk_ms, bk_n = stages["buckets"]
    bk_avg_ms = bk_ms / max(bk_n, 1)
    bk_bytes = 24.0 * st["kmers"] + 4.0 * list_entries
    bk_ach = bk_bytes / (bk_avg_ms * 1e-3) / 1e9 if bk_avg_ms > 0 else 0.0
    bk_traffic, bk_src = pmc_traffic(("part_bounds_kernel", "part_build_kernel<1024", "part_build_kernel<2048", "part_build_kernel<4096"))
    roofline = {"bound": "hbm", "achieved": round(bk_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(bk_ach / HBM_PEAK_GBS, 4), "traffic": bk_traffic,
                "kernel": "bucket build: part_bounds + part_build<1024|2048|4096>",
                "launch_ms": round(bk_avg_ms, 4), "algorithmic_bytes_per_launch": int(bk_bytes),
                "traffic_source": bk_src}
    # the candidate counter itself (the metric's unit is its work):
    # per k-mer 8 B (record) + 4 B per role pair (partner id) + 12 B per dispatched pair
    pc_ms, pc_n = stages["pairs"]
    pc_avg_ms = pc_ms / max(pc_n, 1)
    alg_bytes = 8.0 * st["kmers"] + 4.0 * st["role_pairs"] + 12.0 * st["dispatched"]
    achieved = alg_bytes / (pc_avg_ms * 1e-3) / 1e9 if pc_avg_ms > 0 else 0.0
    traffic, tsrc = pmc_traffic(("pair_count_kernel<false",))
    roofline_pc = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                   "kernel": "pair_count_kernel<false, 256>", "launch_ms": round(pc_avg_ms, 4),
                   "algorithmic_bytes_per_launch": int(alg_bytes), "traffic_source": tsrc}

    # ---- CPU baseline: the C oracle (port of the reference), 1 thread -----
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        n_s = args.cpu_sample_reads
        G_s = int(n_s * args.len / args.coverage)
        b_s, o_s = synth_workload(n_s, args.len, G_s, args.gc, seed=1)
        s = oracle.default_settings(kmer_size=args.k)
        t0 = time.perf_counter()
        r = oracle.Run(packed=(b_s.tobytes(), o_s), settings=s, wide=True, skip_align=True)
        t_cpu = time.perf_counter() - t0
        # role pairs of the sample counted exactly as the GPU counts them
        ovs = sao.Overlapper(kmer_size=args.k, id_mode=sao.SA_IDS_WIDE)
        ovs.add_packed(b_s.tobytes(), o_s)
        ovs.build()
        rp_s = ovs.stats()["role_pairs"]
        assert len(r.lead) == ovs.stats()["dispatched"], "CPU/GPU candidate mismatch on the baseline sample"
        ovs.close()
        cpu = {"value": round(rp_s / t_cpu, 1), "unit": "candidate k-mer pairs/s", "cores": 1, "kind": "port",
               "sample": "%d reads x %d bp, %d bp genome (same 20x coverage), k=%d, hash stage "
                         "(KmerTable.calcPairData+calcDispatchData restated in C, wide ids), %.1f s"
                         % (n_s, args.len, G_s, args.k, t_cpu)}

    if rank == 0:
        line = {
            "metric": "candidate k-mer pairs/sec (hash stage) + aligned read-pairs/sec, k=15, 500 bp reads",
            "value": round(value, 1),
            "unit": "candidate k-mer pairs/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_build / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (splitmix64 genome, error-free 500 bp reads)",
            "config": {"workload": "configs[1]: %dk synthetic %s bp reads/GPU, k=%d, bucket build + "
                                   "edge/middle pair filter" % (args.reads // 1000, (
                                       "%d" % args.len if args.min_len is None else
                                       "%d-%d" % (args.min_len, args.len)), args.k),
                       "reads_per_gpu": args.reads, "read_len": args.len, "min_len": args.min_len, "k": args.k,
                       "genome_bp_per_gpu": G, "ids": "wide",
                       "parallelism": ("sharded-a2a-%s" % args.dist_backend if sharded else
                                       "replicas" if ws > 1 else "single")},
            "aligned_read_pairs_per_s": round(aligned_total / t_align, 1),
            "ms_per_align_step": round(t_align / asteps * 1e3, 3),
            "per_gpu": {k: int(v) for k, v in st.items() if k not in ("aligned", "ovl_records", "dp_cells")},
            "dp_cells_per_align_step": int(ast["dp_cells"]),
            "stage_ms_per_step": {k: round(v[0] / max(args.steps, 1), 4) for k, v in stages.items() if v[1]},
            "align_kernel_ms": round(astages["align"][0] / max(astages["align"][1], 1), 4),
            "quadratic_align": quad,
            "roofline": roofline,
            "roofline_pair_count": roofline_pc,
            "exchange_bytes_per_step_rank0": int(xbytes) if sharded else None,
            "read_allgather_ms": round(t_gather * 1e3, 3) if t_gather is not None else None,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ov.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
