"""Per-kernel time of the timed training steps in a rocprofv3 kernel-trace
database (rocpd sqlite): the steps are the windows between consecutive fused
optimizer kernels (``opt_k``) holding a plausible number of kernels, so
warm-up / capture / guard / post-run work is excluded.

    python tools/step_kernels.py D/.../x_results.db --min 480 --max 520
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--min", type=int, default=480, help="fewest kernels of a training step")
    ap.add_argument("--max", type=int, default=520, help="most kernels of a training step")
    ap.add_argument("--marker", default="opt_k")
    ap.add_argument("--top", type=int, default=80)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("""select d.start, d.end, s.display_name from rocpd_kernel_dispatch d
                          join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start""").fetchall()
    ends = [i for i, r in enumerate(rows) if a.marker in r[2]]
    wins = [(x, y) for x, y in zip(ends[:-1], ends[1:]) if a.min <= y - x <= a.max]
    if not wins:
        raise SystemExit("no step windows")
    agg = defaultdict(lambda: [0, 0])
    tot = span = 0
    for x, y in wins:
        span += rows[y][1] - rows[x][1]
        for st, en, nm in rows[x + 1:y + 1]:
            agg[nm][0] += en - st
            agg[nm][1] += 1
            tot += en - st
    n = len(wins)
    print(f"# {n} steps: {span / n / 1e6:.3f} ms wall per step, {tot / n / 1e6:.3f} ms kernel time, "
          f"{sum(v[1] for v in agg.values()) / n:.0f} kernels per step")
    print("#  ms/step  calls/step  avg_us  kernel")
    for nm, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{t / n / 1e6:9.3f} {c / n:8.1f} {t / c / 1e3:8.1f}  {nm[:110]}")


if __name__ == "__main__":
    main()
