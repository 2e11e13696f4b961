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

Multi-GPU: the sharded context of libsa_overlap
(include/sa_overlap.h, multi.cpp) -- local k-mer emit, RCCL all-to-all of the
records to the shard owning their hash range, bucket build + partial pair
counts there, RCCL all-to-all of the partials to the shard owning the lead,
reduce + collision filter; the packed reads are all-gathered once for the
alignment of each shard's own leads.  Weak scaling: the genome grows with the
GPU count (20x coverage kept) and every GPU holds 100,000 reads of it.
  torchrun --nproc-per-node N bench.py --gpus N   one process per GPU
      (sa_ctx_create_rank; the RCCL unique id and the barrier / max-over-ranks
      timing go over a gloo process group on the host);
  bench.py --gpus N                              one process driving devices
      0..N-1 (sa_ctx_create_multi), one host thread per device.
`value` sums the role pairs over all GPUs.  `--shards S` runs S virtual shards
on one GPU (the exchanges as device copies); `--replicas` (torchrun) runs
independent per-rank datasets with no exchange, for comparison.
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


def synth_genome(genome_len, gc, seed):
    """Base i from splitmix64(seed) output i + 1: G/C with probability gc (then the
    low bit picks G or C), else T/A (oracle.synth_genome is the same in C)."""
    with np.errstate(over="ignore"):
        z = splitmix64(seed, genome_len)
        u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
        bit = (z & np.uint64(1)).astype(np.uint8)
        return np.where(u < gc, np.where(bit == 1, ord("G"), ord("C")),
                        np.where(bit == 1, ord("T"), ord("A"))).astype(np.uint8)


def synth_layout(n_reads, read_len, genome_len, seed, shard=0, min_len=None):
    """Read starts (uniform in [0, G - L], splitmix64((seed ^ 0xABCDEF) + 7919 *
    shard)) and lengths (synth_lengths)."""
    lens = synth_lengths(n_reads, read_len, min_len, seed, shard)
    with np.errstate(over="ignore"):
        rs = (seed ^ 0xABCDEF) + 7919 * shard
        starts = (splitmix64(rs, n_reads) % (np.uint64(genome_len + 1) - lens.astype(np.uint64))).astype(np.int64)
    return starts, lens


def synth_workload(n_reads, read_len, genome_len, gc, seed, shard=0, min_len=None, genome=None):
    """Genome: synth_genome(seed); reads start uniformly in [0, G-L]
    (splitmix64((seed ^ 0xABCDEF) + 7919 * shard): shard r of a multi-GPU run
    samples its own reads of the same genome), forward strand, error-free;
    lengths from synth_lengths.  Returns (bases, offsets)."""
    if genome is None:
        genome = synth_genome(genome_len, gc, seed)
    starts, lens = synth_layout(n_reads, read_len, genome_len, seed, shard, min_len)
    if os.environ.get("SA_BENCH_SORTED_READS") == "1" and lens.min() == lens.max():
        # (experiment only, never the metric's workload: each shard's reads in genome order,
        # i.e. read ids already in locality order -- DESIGN.md 8, item 1)
        starts = np.sort(starts)
    offsets = np.zeros(n_reads + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum(lens)
    # each read is the first len bases of a read_len window at its start (the
    # genome padded so every window exists); chunks of reads bound host memory
    win = np.lib.stride_tricks.sliding_window_view(np.concatenate([genome, np.zeros(read_len, np.uint8)]),
                                                   read_len)
    out = np.empty(int(offsets[-1]), dtype=np.uint8)
    uniform = lens.min() == lens.max()
    keep = np.arange(read_len, dtype=np.int64)[None, :]
    for r0 in range(0, n_reads, 1 << 19):
        r1 = min(n_reads, r0 + (1 << 19))
        if uniform:
            out[int(offsets[r0]):int(offsets[r1])] = win[starts[r0:r1]][:, :read_len].reshape(-1)
        else:
            out[int(offsets[r0]):int(offsets[r1])] = win[starts[r0:r1]][keep < lens[r0:r1, None]]
    return out, offsets


def end_to_end(sao, fasta_path, k, reps=5, cli=None):
    """calc-overlaps from host FASTA bytes to a written .ovl (SURVEY.md 8(d) timing
    protocol; Project4.scala:56-60 -> :795-825) through the C ABI, each repetition
    on a fresh context in this (HIP-initialised) process: median of `reps` of the
    total and of each part -- ctx create, FASTA parse (readSeq), the build
    (upload = read metadata + H2D, the device stages, the strict Trove replay,
    dispatch D2H), the alignment (device, alignment D2H, .ovl formatting) and the
    file write -- the parts from the library's own stage clocks (device stages:
    HIP events; host stages: wall clock).  With `cli`, the sa-overlap process's
    wall time on the same file too (process start and HIP initialisation
    included)."""
    import subprocess
    import tempfile
    runs = []
    out = os.path.join(tempfile.gettempdir(), "sa_e2e_%d.ovl" % os.getpid())
    ovl = b""
    for _ in range(reps):
        r = {}
        t0 = time.perf_counter()
        ov = sao.Overlapper(kmer_size=k, timing=True)
        r["ctx_create"] = time.perf_counter() - t0
        t1 = time.perf_counter()
        ov.read_fasta(fasta_path)
        r["fasta_parse"] = time.perf_counter() - t1
        t1 = time.perf_counter()
        ov.build()
        r["build"] = time.perf_counter() - t1
        t1 = time.perf_counter()
        ov.align()
        r["align"] = time.perf_counter() - t1
        t1 = time.perf_counter()
        ov.write_ovl(out)
        r["write"] = time.perf_counter() - t1
        r["total"] = time.perf_counter() - t0
        st = ov.stage_times()
        for name, (ms, n) in st.items():
            if n:
                r["stage_" + name] = ms / 1e3
        stats = ov.stats()
        ov.close()
        runs.append(r)
    ovl = open(out, "rb").read()
    os.unlink(out)
    keys = sorted({k_ for r in runs for k_ in r})
    med = {k_: float(np.median([r.get(k_, 0.0) for r in runs])) for k_ in keys}
    res = {"total_s": round(med["total"], 4), "reps": reps,
           "breakdown_ms": {k_: round(v * 1e3, 3) for k_, v in med.items() if k_ != "total"},
           "id_mode": "strict" if stats["id_mode"] == sao.SA_IDS_STRICT else "wide",
           "dispatched": int(stats["dispatched"]), "ovl_records": int(stats["ovl_records"]), "ovl_bytes": len(ovl)}
    if cli:
        t0 = time.perf_counter()
        rc = subprocess.run([cli, "-i", fasta_path, "-o", out, "-k", str(k)], capture_output=True, timeout=600)
        res["cli_wall_s"] = round(time.perf_counter() - t0, 3)
        res["cli_identical"] = rc.returncode == 0 and open(out, "rb").read() == ovl
        if os.path.exists(out):
            os.unlink(out)
    return res, ovl


def write_fasta(path, bases, offsets):
    """Reads as FASTA (one line each, headers r1..rN): readSeq's input format."""
    with open(path, "wb") as f:
        b = memoryview(bases)
        for i in range(len(offsets) - 1):
            f.write(b">r%d\n" % (i + 1))
            f.write(b[int(offsets[i]):int(offsets[i + 1])])
            f.write(b"\n")


DEFAULT_WORKLOAD = "n100000_L500_k15"


def workload_label(reads, read_len, min_len, k, n_gpus, mode):
    """config.workload: which BASELINE.json config (or which per-GPU slice of one)
    this shape is, from the shape itself."""
    shape = "%s synthetic %s bp reads/GPU, k=%d" % (
        "%gM" % (reads / 1e6) if reads >= 1000000 else "%dk" % (reads // 1000),
        "%d" % read_len if min_len is None else "%d-%d" % (min_len, read_len), k)
    uniform500 = min_len is None and read_len == 500
    mixed = min_len == 100 and read_len == 1000
    if uniform500 and k == 15 and reads == 100000:
        what = "configs[1]" if n_gpus == 1 else "configs[1] weak-scaled to %d GPUs" % n_gpus
        return "%s: %s, bucket build + edge/middle pair filter" % (what, shape)
    if uniform500 and k == 15 and reads == 1250000:
        return "configs[3] per-GPU slice (10M reads / 8 GPUs) on %s: %s" % (
            "one GPU" if mode == "single" else mode, shape)
    if mixed and k in (12, 15) and reads == 6250000:
        return "configs[4] per-GPU slice (50M reads / 8 GPUs), k=%d pass: %s" % (k, shape)
    if mixed and k in (12, 15):
        return "configs[4]-shaped (mixed 100-1000 bp, k=%d pass), not its size: %s" % (k, shape)
    return "custom shape (not a BASELINE config): %s" % shape


def workload_tag(reads, read_len, min_len, k, gc=0.50, shards=1):
    """Key of a PMC summary: the workload its rocprofv3 passes ran (reads, read
    length(s), k, and GC / virtual shards when not the default)."""
    t = "n%d_L%s_k%d" % (reads, "%d" % read_len if min_len is None else "%d-%d" % (min_len, read_len), k)
    if abs(gc - 0.50) > 1e-9:
        t += "_gc%g" % gc
    if shards > 1:
        t += "_s%d" % shards
    return t


def pmc_summary(tag):
    """Per-kernel counter averages of the newest committed PMC summary of THIS
    workload: profiles/<round>/pmc_summary*__<tag>.csv (tools/prof/profile.sh /
    tools/prof/slice_prof.sh write them from separate rocprofv3 --pmc passes of this
    bench).  Summaries without a tag are the default bench workload's
    (rounds 1-2).  No summary of the workload -> ({}, None): the traffic and
    VALU fields are then null rather than another workload's counters."""
    import csv
    import glob

    def natural(path):  # r02 after r01, pmc_summary_v9 < pmc_summary_v10
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", path)]

    def tag_of(path):
        base = os.path.basename(path)[:-4]
        return base.split("__", 1)[1] if "__" in base else DEFAULT_WORKLOAD
    # any depth under profiles/ (profiles/r03/v1/..., profiles/r03/slices_v2/c3/...); newest by
    # round, then version, in natural order of the path
    files = sorted((f for f in glob.glob(os.path.join(ROOT, "profiles", "**", "pmc_summary*.csv"), recursive=True)
                    if tag_of(f) == tag), key=lambda f: natural(os.path.relpath(f, ROOT)))
    if not files:
        return {}, None
    with open(files[-1]) as f:
        rows = {r["kernel"]: r for r in csv.DictReader(f)}
    return rows, os.path.relpath(files[-1], ROOT)


def isa_mix():
    """The aligner hot loops' VALU mix priced with measured issue costs
    (newest profiles/<round>/isa_mix*.json, written by tools/isa_mix.py)."""
    import glob

    def natural(path):
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", path)]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "isa_mix*.json")), key=natural)
    if not files:
        return None, None
    return json.load(open(files[-1])), os.path.relpath(files[-1], ROOT)


def pmc_sum(rows, kernels, col):
    """Sum over the named kernels (name prefixes) of one counter's per-dispatch
    average; None if a kernel or the counter is missing."""
    tot = 0.0
    for kname in kernels:
        hit = [r for k, r in rows.items() if k.startswith(kname) and r.get(col)]
        if not hit:
            return None
        tot += float(hit[0][col])
    return tot


def hbm_traffic(rows, kernels):
    """HBM bytes per launch of the named kernels from the PMC passes, corrected
    as MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE reports half the
    bytes of coalesced streaming reads on gfx950 (x2), WRITE_SIZE as is (both in
    KiB).  Raw values kept beside it: these kernels' accesses are 8-byte records
    and 4-byte gathers, which the guide leaves uncalibrated."""
    f = pmc_sum(rows, kernels, "FETCH_SIZE_avg")
    w = pmc_sum(rows, kernels, "WRITE_SIZE_avg")
    if f is None or w is None:
        return None, None, None
    return int((2 * f + w) * 1024), int(f * 1024), int(w * 1024)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def note(msg):
    """Progress on stderr (long runs keep their log growing)."""
    print("[bench %.1fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


T_START = time.perf_counter()


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
    ap.add_argument("--replicas", action="store_true", help="torchrun: independent per-rank datasets, no exchange")
    ap.add_argument("--shards", type=int, default=1, help="virtual shards on one GPU (sharded path, device copies)")
    ap.add_argument("--dispatch-hash", action="store_true",
                    help="add a checksum of the dispatch list (lead, trail, count) to the line (cross-build checks)")
    ap.add_argument("--serial-shards", action="store_true",
                    help="virtual shards: run the shards one after another (clean per-shard stage times)")
    ap.add_argument("--lean", action="store_true",
                    help="sharded: SA_OPT_LEAN_MEMORY (free scratch between stages; virtual shards of a "
                         "configs[3]-sized read set on one GPU)")
    ap.add_argument("--pass-budget-mb", type=int, default=0,
                    help="sharded: SA_OPT_PASS_BUDGET_MB (partials per shard and lead-range pass; 0 = from "
                         "the free device memory)")
    ap.add_argument("--stage-steps", type=int, default=5,
                    help="steps of a second, instrumented loop (HIP events around every stage) for the stage "
                         "times and the rooflines; the timed loop itself runs without events")
    ap.add_argument("--check-shards", type=int, default=0,
                    help="single mode: afterwards rebuild the same reads over S virtual shards and require the "
                         "identical dispatch (a size-independent parity property at full size)")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    if ws > 1 and args.gpus not in (1, ws):
        sys.exit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, ws))
    n_gpus = ws if ws > 1 else args.gpus
    # rank: one process per GPU (torchrun); process: one process over n_gpus
    # devices; virtual: --shards on one GPU; replicas / single: no exchange
    mode = ("replicas" if args.replicas else "rank") if ws > 1 else (
        "process" if args.gpus > 1 else "virtual" if args.shards > 1 else "single")
    dist = None
    if ws > 1:
        import torch
        import torch.distributed as dist_
        dist = dist_
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        # host-side group: RCCL unique id broadcast, barriers, max-over-ranks
        # timing; the data path's collectives are RCCL inside libsa_overlap
        dist.init_process_group("gloo")

    import saoverlap as sao

    mean_len = args.len if args.min_len is None else (args.len + args.min_len) / 2.0
    G = int(args.reads * mean_len / args.coverage)
    common = dict(timing=True, kmer_size=args.k, id_mode=sao.SA_IDS_WIDE, align_kernel=args.align_kernel)
    sharded = mode in ("rank", "process", "virtual")
    if mode == "rank":
        # one genome for all ranks (G per GPU, weak scaling); rank r's reads are
        # global ids r*reads+1 .. (r+1)*reads
        bases, offsets = synth_workload(args.reads, args.len, G * ws, args.gc, seed=1, shard=rank,
                                        min_len=args.min_len)
        uid = [sao.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ov = sao.Overlapper(device=local, rank=rank, nranks=ws, rccl_id=uid[0], lean_memory=args.lean,
                            pass_budget_mb=args.pass_budget_mb, **common)
        ov.add_packed(bases.tobytes(), offsets)
    elif mode in ("process", "virtual"):
        P = n_gpus if mode == "process" else args.shards
        ov = sao.Overlapper(gpus=n_gpus, shards=P, serial_shards=args.serial_shards, lean_memory=args.lean,
                            pass_budget_mb=args.pass_budget_mb, **common)
        for r in range(P):  # the same reads the torchrun ranks would hold, in rank order
            b_r, o_r = synth_workload(args.reads, args.len, G * P, args.gc, seed=1, shard=r, min_len=args.min_len)
            ov.add_packed(b_r.tobytes(), o_r)
    else:
        bases, offsets = synth_workload(args.reads, args.len, G, args.gc, seed=1 + rank, min_len=args.min_len)
        ov = sao.Overlapper(device=local if ws > 1 else 0, **common)
        ov.add_packed(bases.tobytes(), offsets)
    if mode in ("process", "virtual"):  # one shard's reads (the per-GPU byte model)
        offsets = np.concatenate([[0], np.cumsum(synth_lengths(args.reads, args.len, args.min_len, 1, 0))])
    build_step = ov.device_build
    tag = workload_tag(args.reads, args.len, args.min_len, args.k, args.gc, args.shards if mode == "virtual" else 1)

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    # ---- hash stage (configs[1]) ------------------------------------------
    note("inputs ready (%d reads)" % (len(offsets) - 1))
    ov.sync()
    t0 = time.perf_counter()
    build_step()  # allocations happen here, outside the timed region
    ov.sync()
    t_first = max_over_ranks(time.perf_counter() - t0)
    note("first build done")
    # the first build after the allocations: what a single CLI run pays, then warm-up
    # (nothing is remembered between builds of one read set except, on the sharded
    # path, its partials / bound ratio -- which a first build estimates with a probe)
    t_second = None
    for i in range(args.warmup):
        ov.sync()
        t0 = time.perf_counter()
        build_step()
        ov.sync()
        if i == 0:
            t_second = max_over_ranks(time.perf_counter() - t0)
    xb0 = ov.exchanged_bytes()
    # the timed loop runs without stage events (each HIP event record is a
    # packet on the stream); a second, instrumented loop gives the stage times
    ov.set_timing(False)
    barrier()
    ov.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        build_step()
    ov.sync()
    barrier()
    t_build = max_over_ranks(time.perf_counter() - t0)
    st = ov.stats()
    xbytes = (ov.exchanged_bytes() - xb0) / max(args.steps, 1)
    stage_steps = max(1, args.stage_steps)
    ov.set_timing(True)
    ov.reset_stage_times()
    barrier()
    ov.sync()
    t0 = time.perf_counter()
    for _ in range(stage_steps):
        build_step()
    ov.sync()
    barrier()
    t_instr = max_over_ranks(time.perf_counter() - t0)
    stages = ov.stage_times()
    role_pairs_total = sum_over_ranks(float(st["role_pairs"])) * args.steps
    value = role_pairs_total / t_build

    note("hash stage timed: %.3f ms/step" % (t_build / args.steps * 1e3))
    # ---- end-to-end incl. banded HOXD alignment (configs[2]) --------------
    asteps = max(1, args.align_steps) if args.align_steps is not None else max(1, args.steps // 2)  # (>= 1: the aligner fields need one timed step)
    # first align of a sharded context all-gathers the packed reads: timed apart
    barrier()
    t0 = time.perf_counter()
    ov.device_align()
    ov.sync()
    barrier()
    t_gather = max_over_ranks(time.perf_counter() - t0) if sharded else None
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

    # ---- rooflines --------------------------------------
    # Units of ONE GPU's share of the step (rank mode: this rank's; one process
    # over P shards: the total / P).  Config-2 byte model: N*L/4 (2-bit packed
    # reads) + 32 B per k-mer occurrence (8 emit write + 16 bucket-build read +
    # write + 8 pairing read) + 16 B per distinct ordered read pair (count write
    # + read); role pairs are aggregated on chip and cost no HBM bytes.
    P_here = 1 if mode in ("rank", "single", "replicas") else (n_gpus if mode == "process" else args.shards)
    kmers_g = st["kmers"] / P_here
    pairs_g = st["pairs"] / P_here
    bases_g = float(offsets[-1])
    step_bytes = bases_g / 4.0 + 32.0 * kmers_g + 16.0 * pairs_g
    rows, pmc_src = pmc_summary(tag)
    ms_step = t_build / args.steps * 1e3

    def roof(bytes_, ms, kernels, name):
        ach = bytes_ / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        tr, fr, wr = hbm_traffic(rows, kernels) if kernels else (None, None, None)
        return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tr, "kernel": name, "launch_ms": round(ms, 4),
                "algorithmic_bytes_per_launch": int(bytes_), "traffic_fetch_raw": fr, "traffic_write_raw": wr,
                "traffic_source": pmc_src if tr is not None else None}

    def per_launch(stage):
        ms_, n_ = stages[stage]
        return ms_ / max(n_, 1)

    # dominant kernel by time: the bucket build (part_bounds + part_build at the
    # 1,024 / 2,048 / 4,096-record tiers + the split tier, one HIP-event scope on
    # the library's stream); 16 B per k-mer in the model
    bk_kernels = ("sa::part_bounds_kernel", "void sa::part_build_kernel<1024", "void sa::part_build_kernel<2048",
                  "void sa::part_build_kernel<4096")
    if any(k.startswith("sa::part_split_kernel") for k in rows):  # (summaries of trees with the split tier)
        bk_kernels += ("sa::part_split_kernel",)
    roofline = roof(16.0 * kmers_g, per_launch("buckets"), bk_kernels,
                    "bucket build: part_bounds + part_build<1024|2048|4096> + part_split")
    # the bucket build runs in one of two per-process modes at the bench shape
    # ("Bucket-build bimodality"): say which one this line hit
    if tag == DEFAULT_WORKLOAD:
        # (round 4: the slow mode moved from 1.31-1.33 to 1.19-1.21 ms with the
        # lists written non-temporally; the fast mode was 1.05-1.15 before that)
        roofline["bucket_build_mode"] = "slow (> 1.1 ms)" if per_launch("buckets") > 1.1 else "fast (<= 1.1 ms)"
    # the first pair-count pass: one wave per read (round 3; wide ids, per-read regions), or
    # the one-read workgroup kernel in profiles of earlier trees / other modes
    pc_k = ("sa::pair_count_wave_kernel",) if any(k.startswith("sa::pair_count_wave_kernel") for k in rows) \
        else ("void sa::pair_count_kernel<false, 256",)
    roofline_pc = roof(8.0 * kmers_g + 16.0 * pairs_g, per_launch("pairs"), pc_k, pc_k[0].split("sa::")[1])
    pc_conf = pmc_sum(rows, pc_k, "SQ_LDS_BANK_CONFLICT_avg")
    pc_act = pmc_sum(rows, pc_k, "SQ_LDS_IDX_ACTIVE_avg")
    roofline_pc["lds_bank_conflict_rate"] = round(pc_conf / pc_act, 4) if pc_conf is not None and pc_act else None
    roofline_step = roof(step_bytes, ms_step, None, "whole hash step (every kernel, wall clock)")
    # the aligner (configs[2]): integer VALU, MFMA unused.  Peak = 256 CUs x 4
    # SIMD-32 x 32 lanes x 2.4 GHz = 78.6 T lane-ops/s (a wave64 VALU op issues
    # over 2 cycles, MI355X_MICROARCH.md).  achieved = measured SQ_INSTS_VALU of
    # the dovetail kernels x 64 lanes / their event time; nominal = SURVEY.md
    # 8(d)'s 18 int32 ops per DP cell.
    VALU_PEAK = 256 * 4 * 32 * 2.4e9 / 1e12
    al_ms = astages["align"][0] / max(astages["align"][1], 1)
    cells_g = ast["dp_cells"] / P_here
    # at the bench shape both phases run two pairs per lane (packed 16-bit halves,
    # DESIGN.md 4.6): one issue slot there does two cells' operation.  The peak is
    # the measured per-instruction issue cost (tools/valu_rate.hip: ~2.55 cycles per
    # wave per SIMD for add/sub/bitwise/bitop3, ~4.35 for v_pk_*, max/min, perm, bfi)
    # over the hot loops' static mix (tools/isa_mix.py): lane-ops/s the SIMDs can
    # issue for THIS instruction mix; the 2-cycle figure stays beside it as nominal.
    mix, mix_src = isa_mix()
    # (phase 1 is dovetail_p1x2_seg_kernel since round 5, dovetail_p1x2_kernel before: one prefix)
    kern = (("sa::dovetail_p1x2_", "dovetail_p1x2"), ("sa::dovetail_p2tbx2_kernel", "dovetail_p2tbx2"))
    valu_k = [pmc_sum(rows, (kn,), "SQ_INSTS_VALU_avg") for kn, _ in kern]
    valu = sum(valu_k) if None not in valu_k else None
    valu_ach = valu * 64 / (al_ms * 1e-3) / 1e12 if valu is not None and al_ms > 0 else None
    mix_peak = None
    if valu is not None and mix and all(m in mix for _, m in kern):
        cyc = sum(v * mix[m]["avg_cycles_per_valu"] for v, (_, m) in zip(valu_k, kern)) / valu
        mix_peak = 1024 * 64 * 2.4e9 / cyc / 1e12
    # frac leads with the nominal gfx950 VALU peak (2 cycles per wave64 op); the
    # mix-weighted peak (measured issue costs of the kernels' own instruction
    # mix) is kept beside it
    roofline_align = {"bound": "valu", "unit": "T lane-ops/s",
                      "peak": round(VALU_PEAK, 1),
                      "achieved": round(valu_ach, 2) if valu_ach is not None else None,
                      "frac": round(valu_ach / VALU_PEAK, 4) if valu_ach is not None else None,
                      "peak_mix_weighted": round(mix_peak, 1) if mix_peak else None,
                      "frac_mix_weighted": round(valu_ach / mix_peak, 4) if valu_ach is not None and mix_peak else None,
                      "mix_source": mix_src,
                      "kernel": "dovetail_p1x2 + dovetail_p2tbx2 (+ phase-2 pair regrouping sort)",
                      "gcups": round(cells_g / (al_ms * 1e-3) / 1e9, 1) if al_ms else None,
                      "launch_ms": round(al_ms, 4), "dp_cells_per_launch": int(cells_g),
                      "nominal_18_ops_per_cell": round(18.0 * cells_g / (al_ms * 1e-3) / 1e12, 2) if al_ms else None,
                      "valu_wave_insts_per_launch": int(valu) if valu is not None else None,
                      "lds_bank_conflict_rate": "n/a: the lane kernels keep the band in registers (no LDS)",
                      "source": pmc_src if valu is not None else None}
    grp_conf = pmc_sum(rows, ("void sa::dovetail_kernel",), "SQ_LDS_BANK_CONFLICT_avg")
    grp_act = pmc_sum(rows, ("void sa::dovetail_kernel",), "SQ_LDS_IDX_ACTIVE_avg")
    if grp_conf is not None and grp_act:
        roofline_align["lds_bank_conflict_rate_group_kernel"] = round(grp_conf / grp_act, 4)

    # ---- CPU baselines (rank 0, N = 1): the C oracle on this box's cores ---
    cpu = None
    config0 = None
    config2_e2e = None
    if rank == 0 and n_gpus == 1 and mode == "single" and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        cores_all = oracle.max_threads()
        n_s = args.cpu_sample_reads
        G_s = int(n_s * args.len / args.coverage)
        b_s, o_s = synth_workload(n_s, args.len, G_s, args.gc, seed=1)
        s = oracle.default_settings(kmer_size=args.k)
        t0 = time.perf_counter()
        r = oracle.Run(packed=(b_s.tobytes(), o_s), settings=s, wide=True, skip_align=True)
        t_cpu = time.perf_counter() - t0
        # the same hash stage on all of this job's cores (OpenMP restatement:
        # per-thread PairData maps over hash bins, merged by lead; same pairs)
        t0 = time.perf_counter()
        r_mt = oracle.Run(packed=(b_s.tobytes(), o_s), settings=s, wide=True, skip_align=True, threads=cores_all)
        t_cpu_mt = time.perf_counter() - t0
        # role pairs of the sample counted exactly as the GPU counts them
        ovs = sao.Overlapper(kmer_size=args.k, id_mode=sao.SA_IDS_WIDE)
        ovs.add_packed(b_s.tobytes(), o_s)
        ovs.build()
        rp_s = ovs.stats()["role_pairs"]
        lead_s, trail_s, _ = ovs.dispatch()
        assert np.array_equal(r.lead, lead_s) and np.array_equal(r.trail, trail_s), \
            "CPU/GPU dispatch mismatch on the baseline sample"
        assert np.array_equal(r_mt.lead, lead_s) and np.array_equal(r_mt.trail, trail_s) and \
            r_mt.role_pairs == rp_s, "all-core CPU / GPU hash stage mismatch on the baseline sample"
        # aligner: the same dispatch (first pairs of it), 1 thread and all threads,
        # each tuple checked against the GPU's
        ovs.align()
        gal = ovs.alignments()
        na1, naa = min(len(lead_s), 20000), min(len(lead_s), 200000)
        b_bytes = b_s.tobytes()
        t0 = time.perf_counter()
        c1 = oracle.align_batch(b_bytes, o_s, lead_s[:na1], trail_s[:na1], settings=s, threads=1)
        t_a1 = time.perf_counter() - t0
        t0 = time.perf_counter()
        ca = oracle.align_batch(b_bytes, o_s, lead_s[:naa], trail_s[:naa], settings=s, threads=0)
        t_aa = time.perf_counter() - t0
        for name in ("start_i", "start_j", "end_i", "end_j", "correct", "error", "ahg", "bhg"):
            assert np.array_equal(ca[:, oracle.ALIGN_FIELDS.index(name)],
                                  gal[:naa, sao.ALIGN_FIELDS.index(name)]), "CPU/GPU alignment mismatch: " + name
        ovs.close()
        cpu = {"value": round(rp_s / t_cpu, 1), "unit": "candidate k-mer pairs/s", "cores": 1, "kind": "port",
               "sample": "%d reads x %d bp, %d bp genome (same 20x coverage), k=%d, hash stage "
                         "(KmerTable.calcPairData + calcDispatchData restated in C, one thread: the reference's "
                         "KmerTable is single-writer), %.1f s; dispatch equal to the GPU's"
                         % (n_s, args.len, G_s, args.k, t_cpu),
               "all_cores": {"value": round(rp_s / t_cpu_mt, 1), "cores": cores_all, "s": round(t_cpu_mt, 2),
                             "sample": "the same sample and stage on %d OpenMP threads (this job's CPU share): "
                                       "per-thread PairData maps over hash bins merged by lead "
                                       "(oracle orc_run_wide_mt); dispatch and role pairs equal to the GPU's"
                                       % cores_all},
               "cpu_model": cpu_model(), "nproc": os.cpu_count(),
               "align": {"unit": "aligned read-pairs/s", "kind": "port",
                         "value_1_thread": round(na1 / t_a1, 1), "value_all_threads": round(naa / t_aa, 1),
                         "threads_all": cores_all,
                         "sample": "first %d / %d dispatched pairs of the sample, generateFastDovetailAlignment"
                                   "Set restated in C (OpenMP over pairs, as genBlockMTAlign's actor pool); "
                                   "%.1f s / %.1f s; tuples equal to the GPU's" % (na1, naa, t_a1, t_aa)}}
        # configs[0]: reconstructed c_ruddii reads (32,000 x 100 bp, ids in .seq
        # order), k = 15, strict ids, whole calc-overlaps path -> .ovl bytes
        z = np.load(os.path.join(ROOT, "tests", "golden", "c_ruddii_layout.npz"))
        contig = z["contig"].tobytes()
        cr = [contig[o:o + 100] for o in z["offset"][1:]]
        t0 = time.perf_counter()
        rc0 = oracle.Run(reads=cr, settings=oracle.default_settings(kmer_size=15))
        t_c0 = time.perf_counter() - t0
        import tempfile
        cli = os.path.join(ROOT, "sequence-aligner_amd", "build", "sa-overlap")
        fa0 = os.path.join(tempfile.gettempdir(), "sa_c_ruddii_%d.seq" % os.getpid())
        cb = b"".join(cr)
        write_fasta(fa0, cb, np.concatenate([[0], np.cumsum([len(x) for x in cr])]))
        e2e0, g_ovl = end_to_end(sao, fa0, 15, reps=5, cli=cli if os.path.exists(cli) else None)
        os.unlink(fa0)
        config0 = {"workload": "configs[0]: c_ruddii reconstructed 32,000 x 100 bp reads, k=15, strict ids, "
                               "FASTA file -> .ovl file",
                   "cpu_port_1_thread_s": round(t_c0, 3), "gpu_end_to_end_s": e2e0["total_s"],
                   "gpu_end_to_end": e2e0,
                   "ovl_records": g_ovl.count(b"{OVL"), "ovl_identical": g_ovl == rc0.ovl}
        # configs[2] end to end: the bench's 100k reads as a FASTA file -> written .ovl
        fa2 = os.path.join(tempfile.gettempdir(), "sa_bench_%d.seq" % os.getpid())
        write_fasta(fa2, bases, offsets)
        e2e2, _ = end_to_end(sao, fa2, args.k, reps=5, cli=cli if os.path.exists(cli) else None)
        os.unlink(fa2)
        config2_e2e = dict(e2e2, workload="configs[2]: %d x %d bp reads (this bench's), k=%d, wide ids, FASTA "
                                           "file -> .ovl file" % (args.reads, args.len, args.k))

    note("aligner timed")
    dhash = None
    if args.dispatch_hash:
        ld, tr, ct = (np.asarray(x, dtype=np.uint64) for x in ov.dispatch())
        w = np.arange(1, len(ld) + 1, dtype=np.uint64)
        with np.errstate(over="ignore"):
            dhash = "%016x" % int(np.bitwise_xor.reduce((ld * np.uint64(0x9E3779B97F4A7C15) + tr * np.uint64(
                0xC2B2AE3D27D4EB4F) + ct * np.uint64(0x165667B19E3779F9)) * w) if len(ld) else 0)
    # ---- full-size parity property: S virtual shards == one device ----------
    check = None
    if args.check_shards > 1 and mode == "single":
        lead1, trail1, cnt1 = (np.array(x) for x in ov.dispatch())
        ov.close()  # its HBM back before the sharded context allocates
        t0 = time.perf_counter()
        check = {"shards": args.check_shards, "dispatched": int(len(lead1))}
        try:
            ovx = sao.Overlapper(shards=args.check_shards, **common)
            ovx.add_packed(bases.tobytes(), offsets)
            ovx.device_build()
            lead2, trail2, cnt2 = ovx.dispatch()
            check["dispatch_identical"] = bool(np.array_equal(lead1, lead2) and np.array_equal(trail1, trail2)
                                               and np.array_equal(cnt1, cnt2))
            check["sharded_build_s"] = round(time.perf_counter() - t0, 3)
            ovx.close()
        except sao.SAError as e:  # e.g. SA_E_NOMEM: the record is kept, the line still printed
            check["error"] = str(e)

    if rank == 0:
        line = {
            "metric": "candidate k-mer pairs/sec (hash stage) + aligned read-pairs/sec, k=15, 500 bp reads",
            "value": round(value, 1),
            "unit": "candidate k-mer pairs/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "first_build_ms": {"incl_allocation": round(t_first * 1e3, 3),
                               "second": round(t_second * 1e3, 3) if t_second is not None else None},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (splitmix64 genome, error-free reads)",
            "config": {"workload": workload_label(args.reads, args.len, args.min_len, args.k, n_gpus, mode),
                       "reads_per_gpu": args.reads, "read_len": args.len, "min_len": args.min_len, "k": args.k,
                       "genome_bp_per_gpu": G, "ids": "wide", "pmc_key": tag,
                       "parallelism": {"rank": "rccl-a2a, one process per GPU", "process":
                                       "rccl-a2a, one process over %d devices" % n_gpus,
                                       "virtual": "%d virtual shards on one GPU" % args.shards,
                                       "replicas": "replicas (no exchange)", "single": "single"}[mode]},
            "aligned_read_pairs_per_s": round(aligned_total / t_align, 1),
            "ms_per_align_step": round(t_align / asteps * 1e3, 3),
            "per_gpu": {k: int(v) for k, v in st.items() if k not in ("aligned", "ovl_records", "dp_cells")},
            "dp_cells_per_align_step": int(ast["dp_cells"]),
            "ms_per_step_instrumented": round(t_instr / stage_steps * 1e3, 3),
            "stage_ms_per_step": {k: round(v[0] / stage_steps, 4) for k, v in stages.items() if v[1]},
            "align_kernel_ms": round(al_ms, 4),
            "quadratic_align": quad,
            "roofline": roofline,
            "roofline_step": roofline_step,
            "roofline_pair_count": roofline_pc,
            "roofline_align": roofline_align,
            "exchange_bytes_per_step": int(xbytes) if sharded else None,
            "shard_info": ov.shard_info() if sharded else None,
            "read_allgather_ms": round(t_gather * 1e3, 3) if t_gather is not None else None,
            "cpu_baseline": cpu,
            "config0": config0,
            "config2_end_to_end": config2_e2e,
            "check_shards": check,
            "dispatch_hash": dhash,
        }
        print(json.dumps(line), flush=True)
    ov.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
