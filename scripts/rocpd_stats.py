"""Kernel statistics (calls, total / average duration, share) from a rocprofv3 SQLite output
(rocpd tables), the summary `--stats` prints as CSV when the output format is CSV.
    python scripts/rocpd_stats.py gpurun_out/prof512/run_results.db [> profiles/...txt]"""
import collections
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    names = {i: (n, v, a) for i, n, v, a in cur.execute(
        f"select id, display_name, arch_vgpr_count, accum_vgpr_count from {ks}")}
    agg = collections.defaultdict(lambda: [0, 0])
    for kid, s, e in cur.execute(f"select kernel_id, start, end from {kd}"):
        agg[kid][0] += 1
        agg[kid][1] += e - s
    total = sum(v[1] for v in agg.values())
    print(f"{'kernel':70s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>9s} {'share':>6s} vgpr")
    for kid, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        name, vg, ag = names[kid]
        print(f"{name[:70]:70s} {n:7d} {t / 1e6:10.2f} {t / n / 1e3:9.2f} {t / total:6.1%} {vg}+{ag}")


if __name__ == "__main__":
    main(sys.argv[1])
