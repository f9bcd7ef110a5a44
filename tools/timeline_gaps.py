"""Idle time between kernels inside training steps, from a rocprofv3
kernel-trace database (rocpd sqlite): per step (delimited by the fused
optimizer kernel ``opt_k``, one per step) the wall span, the time covered by
at least one kernel, the idle remainder, the number of kernels, and the
(previous kernel -> next kernel) pairs with the most idle time between them.
Answers "how much of the step is launch / dependency gaps" for a captured or
eager step.

    rocprofv3 --kernel-trace -d D -o x --output-format rocpd -- python3 bench.py --steps 6 --warmup 3
    python tools/timeline_gaps.py D/.../x_results.db --last 4
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str, n: int = 60) -> str:
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)", name)
    s = m.group(1) if m else name
    return s[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=4, help="analyse the last N complete steps")
    ap.add_argument("--marker", default="opt_k", help="kernel name substring that ends a step")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--min-kernels", type=int, default=50)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("""select d.start, d.end, s.display_name from rocpd_kernel_dispatch d
                          join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start""").fetchall()
    ends = []
    for i, r in enumerate(rows):  # (marker kernels closer than --min-kernels apart: not a training step)
        if a.marker in r[2] and (not ends or i - ends[-1] >= a.min_kernels):
            ends.append(i)
    if len(ends) < 2:
        raise SystemExit(f"fewer than two '{a.marker}' kernels: cannot delimit steps")
    ends = ends[-(a.last + 1):]
    pair_idle = defaultdict(lambda: [0, 0])
    tot_span = tot_busy = 0
    nsteps = 0
    for s0, s1 in zip(ends[:-1], ends[1:]):
        ks = rows[s0 + 1:s1 + 1]
        t0 = rows[s0][1]  # the previous step's optimizer end
        t1 = ks[-1][1]
        busy = 0
        cur_s, cur_e = None, None
        prev_name = rows[s0][2]
        for st, en, nm in ks:
            if cur_e is None or st > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                gap = st - (cur_e if cur_e is not None else t0)
                if gap > 0:
                    pi = pair_idle[(short(prev_name), short(nm))]
                    pi[0] += gap
                    pi[1] += 1
                cur_s, cur_e = st, en
            else:
                cur_e = max(cur_e, en)
            prev_name = nm
        busy += cur_e - cur_s
        span = t1 - t0
        tot_span += span
        tot_busy += busy
        nsteps += 1
        print(f"step: span {span / 1e6:8.3f} ms  busy {busy / 1e6:8.3f} ms  idle {(span - busy) / 1e6:7.3f} ms "
              f"({100 * (span - busy) / span:5.2f} %)  kernels {len(ks)}")
    print(f"# mean over {nsteps} steps: span {tot_span / nsteps / 1e6:.3f} ms, idle {(tot_span - tot_busy) / nsteps / 1e6:.3f} ms "
          f"({100 * (tot_span - tot_busy) / tot_span:.2f} %)")
    print("# idle per step by (previous kernel -> next kernel), largest first")
    for (p, n), (t, c) in sorted(pair_idle.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{t / 1e3 / nsteps:9.1f} us/step {c / nsteps:6.1f}x  {p}  ->  {n}")


if __name__ == "__main__":
    main()
