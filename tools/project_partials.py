"""Projection of the sharded count's per-rank partials at a BASELINE config's real
density: sampled leads of the config's own read set, counted
by the oracle (orc_lead_stats -- CPU, test infrastructure) over reads cut from the
config's genome without materialising them.

Per sampled lead: distinct partners (PairData rows with that fst), role pairs as fst,
partials over P = 8 hash-range owners (distinct (partner, owner of the k-mer): what the
8 ranks' pair counters write for that lead in all, KmerTable.scala:85-149 per owner)
and dispatched partners ([min, max] = [7, 222]).  Leads are uniform over the reads, so
N x the sample means estimate the totals; each rank counts 1/P of them (owners by a
hash of the k-mer) and reduces the partials of its own N/P leads.

  python tools/project_partials.py c3            # configs[3]: 10M x 500 bp, 250 Mbp, k=15
  python tools/project_partials.py c4 --k 15     # configs[4]: 50M x 100-1000 bp, 1.375 Gbp
  python tools/project_partials.py c4 --k 12 --leads 300
Writes profiles/r06/projection/<config>_k<k>.json.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402
import oracle  # noqa: E402

# configs[3] G = 250 Mbp seed 4; configs[4] G = 1.375 Gbp seed 5
CONFIGS = {
    "c3": dict(reads=10_000_000, len=500, min_len=None, genome=250_000_000, seed=4, k=15),
    "c4": dict(reads=50_000_000, len=1000, min_len=100, genome=1_375_000_000, seed=5, k=15),
    # the sizes the GPU tests run, for the projection's own check against measured partials
    "c3test": dict(reads=10_000_000, len=500, min_len=None, genome=250_000_000, seed=4, k=15),
}

# per partial entry and rank: pair-counter regions (5/4 of 12 B), send 12 B, receive
# 12 B, reduce scratch ~28 B (multi.cpp pass_budget)
BYTES_PER_PARTIAL_RANK = 15 + 12 + 12 + 28


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=sorted(CONFIGS))
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--leads", type=int, default=2000)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06", "projection"))
    a = ap.parse_args()
    cfg = dict(CONFIGS[a.config])
    if a.k:
        cfg["k"] = a.k
    n, P = cfg["reads"], a.ranks
    log_ranks = P.bit_length() - 1
    t0 = time.time()
    genome = oracle.synth_genome(cfg["seed"], cfg["genome"], 0.5, a.threads)
    starts, lens = bench.synth_layout(n, cfg["len"], cfg["genome"], cfg["seed"], 0, cfg["min_len"])
    t_gen = time.time() - t0
    rng = np.random.default_rng(11)
    leads = np.unique(rng.integers(1, n + 1, a.leads)).astype(np.int32)
    s = oracle.default_settings(kmer_size=cfg["k"])
    t0 = time.time()
    st = oracle.lead_stats(genome, starts, lens.astype(np.int32), leads, settings=s, threads=a.threads,
                           log_ranks=log_ranks)
    t_orc = time.time() - t0
    mean = st.mean(axis=0)
    sem = st.std(axis=0, ddof=1) / np.sqrt(len(leads))
    kmers = int(np.clip(lens - cfg["k"] + 1, 0, None).sum())
    tot = {name: float(mean[i] * n) for i, name in enumerate(("distinct_pairs", "role_pairs", "partials",
                                                              "dispatched"))}
    per_rank_partials = tot["partials"] / P
    out = {
        "config": a.config, "reads": n, "read_len": cfg["len"], "min_len": cfg["min_len"], "genome_bp": cfg["genome"],
        "seed": cfg["seed"], "k": cfg["k"], "ranks": P, "kmers": kmers, "kmers_per_rank": kmers / P,
        "sampled_leads": int(len(leads)),
        "per_lead_mean": {"distinct_partners": mean[0], "role_pairs": mean[1], "partials": mean[2],
                          "dispatched": mean[3]},
        "per_lead_sem": {"distinct_partners": sem[0], "role_pairs": sem[1], "partials": sem[2], "dispatched": sem[3]},
        "per_lead_max": {"distinct_partners": int(st[:, 0].max()), "partials": int(st[:, 2].max())},
        "projected_total": tot,
        "projected_per_rank": {
            "partials": per_rank_partials,
            "partial_bytes": per_rank_partials * 12,
            "exchange2_bytes_sent": per_rank_partials * 12 * (P - 1) / P,
            "exchange1_bytes_sent": kmers / P * 8 * (P - 1) / P,
            "single_pass_hbm_bytes": per_rank_partials * BYTES_PER_PARTIAL_RANK,
            "received_records": kmers / P,
        },
        "seconds": {"generate": round(t_gen, 1), "oracle": round(t_orc, 1)},
        "note": "oracle orc_lead_stats over sampled leads (uniform over read ids) of the config's own read set; "
                "totals = reads x sample mean; per rank = total / ranks (owners by k-mer hash)",
    }
    os.makedirs(a.out, exist_ok=True)
    path = os.path.join(a.out, "%s_k%d.json" % (a.config, cfg["k"]))
    with open(path, "w") as f:
        json.dump(out, f, indent=1, default=float)
    print(json.dumps(out, default=float))


if __name__ == "__main__":
    main()
