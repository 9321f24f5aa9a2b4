"""Per-kernel summary (calls, average/min/max microseconds) from a rocprofv3
rocpd SQLite output (rocprofv3 -d DIR -o NAME writes DIR/**/NAME_results.db).

usage: python tools/prof_db_stats.py DB [substring ...]"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    keys = sys.argv[2:]
    c = sqlite3.connect(db)
    agg = collections.OrderedDict()
    for name, start, end, grid in c.execute("select name, start, end, grid_x from kernels order by start"):
        k = name.split("(")[0]
        if keys and not any(s in k for s in keys):
            continue
        agg.setdefault((k, grid), []).append((end - start) / 1e3)
    print(f"{'kernel':28s} {'grid':>9s} {'calls':>5s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s}")
    for (k, grid), v in agg.items():
        print(f"{k:28s} {grid:9d} {len(v):5d} {sum(v) / len(v):10.1f} {min(v):10.1f} {max(v):10.1f}")


if __name__ == "__main__":
    main()
