"""Per-launch extracts of a round's bench kernel trace (measurement aid).

usage: round_extracts.py TRACE_CSV[.gz] TAG
Writes, from the rocprofv3 kernel trace of `python3 bench.py --no-traffic --no-cpu-baseline`
(scripts/gpu_round.sh):
  profiles/<TAG>_pr_launches.csv       every PageRank push / apply launch (make_profile_md.py
                                       drops the post-convergence no-op launches from it)
  profiles/<TAG>_louvain_launches.md   Louvain heavy-row (k_big_*) and hash-sweep launches per
                                       leg: the legs are the bench's last two graphs (RMAT-23,
                                       then RMAT-26), told apart by their k_rmat launches
  profiles/<TAG>_sssp_kernels.md       the SSSP leg's kernels (between its graph's k_rmat and the
                                       next one)
"""
import csv
import gzip
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_summary import short  # noqa: E402


def load(path):
    f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        r["_n"] = short(r["Kernel_Name"])
        r["_d"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return rows


def table(rows, names, title):
    out = [f"### {title}", "", "| kernel | launches | mean µs | median µs | max µs | total ms |", "|---|---|---|---|---|---|"]
    for n in names:
        d = [r["_d"] / 1e3 for r in rows if r["_n"] == n]
        if d:
            out.append(f"| `{n}` | {len(d)} | {statistics.mean(d):.1f} | {statistics.median(d):.1f} | {max(d):.1f} | "
                       f"{sum(d) / 1e3:.2f} |")
    return out + [""]


def main():
    path, tag = sys.argv[1], sys.argv[2]
    rows = load(path)
    with open(f"profiles/{tag}_pr_launches.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "duration_ns"])
        for r in rows:
            if r["_n"].startswith("k_pr_push") or r["_n"] == "k_pr_apply":
                w.writerow([r["_n"], r["_d"]])
    # graph generations of the legs (the tiny calibration / warm-up graphs' k_rmat run in µs)
    rm = [i for i, r in enumerate(rows) if r["_n"] == "k_rmat" and r["_d"] > 500_000]
    big = ["k_big_partials", "k_big_buckets", "k_big_move", "k_sweep_hash", "k_sweep_hash_wide"]
    out = [f"# Louvain launches, round {tag} (`{path.rsplit('/', 1)[-1]}`)", "",
           "Per-launch durations from the rocprofv3 kernel trace of the bench (every level and",
           "sweep of every timed and warm-up call of the leg).", ""]
    if len(rm) >= 2:
        out += table(rows[rm[-2]:rm[-1]], big, "RMAT-23 leg (configs[5]-sized, one GPU)")
        out += table(rows[rm[-1]:], big, "RMAT-26 leg (configs[4]'s graph, one GPU)")
    open(f"profiles/{tag}_louvain_launches.md", "w").write("\n".join(out) + "\n")
    # the SSSP leg: the graph whose segment holds k_relax launches
    segs = list(zip(rm, rm[1:] + [len(rows)]))
    ss = [(a, b) for a, b in segs if any(r["_n"] == "k_relax" for r in rows[a:b])]
    if ss:
        a, b = ss[0]
        names = {}
        for r in rows[a:b]:
            names[r["_n"]] = names.get(r["_n"], 0) + r["_d"]
        top = [n for n, _ in sorted(names.items(), key=lambda x: -x[1])[:14]]
        out = [f"# SSSP leg kernels, round {tag}", ""] + table(rows[a:b], top, "RMAT-24, uniform weights (graph build included)")
        open(f"profiles/{tag}_sssp_kernels.md", "w").write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
