"""List the dispatches of kernels matching a pattern from a rocprofv3 rocpd
database: grid size, workgroup size, LDS and duration, grouped by grid (one
line per distinct launch shape, with count and mean time) -- which layer
shapes a generic kernel serves.

    python tools/kernel_dispatches.py DB 'igemm_k<128, 128, 0, 0, 0, 256, 2, 2, 1, 0>' [--steps 11]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("pattern")
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type in ('table','view')")]
    kt = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in cur.execute(f"pragma table_info({kt})")]
    gx = next(c for c in cols if c.startswith("grid_size_x") or c == "grid_size_x")
    q = (f"select s.display_name, k.{gx}, k.grid_size_y, k.grid_size_z, k.workgroup_size_x, k.end - k.start "
         f"from {kt} k join {ks} s on k.kernel_id = s.id")
    g = defaultdict(list)
    for name, x, y, z, wg, dur in cur.execute(q):
        if a.pattern in name:
            g[(x // max(wg, 1), y, z)].append(dur)
    tot = 0.0
    for key, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        tot += sum(v)
        print(f"grid(wg)={key}  calls/step={len(v) / a.steps:.1f}  mean_us={sum(v) / len(v) / 1e3:.1f}  "
              f"ms/step={sum(v) / a.steps / 1e6:.3f}")
    print(f"total ms/step {tot / a.steps / 1e6:.3f}")


if __name__ == "__main__":
    main()
