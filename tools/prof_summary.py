"""Per-kernel summary of a rocprofv3 database (rocpd sqlite written by
``rocprofv3 --kernel-trace -d DIR -o NAME``): total / per-step ms, share,
calls, average us, VGPR/AGPR/LDS per kernel.

    python tools/prof_summary.py gpurun_out/prof/r50_results.db --steps 8 > profiles/x.txt
"""
import argparse
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=float, default=1.0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--width", type=int, default=110)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("""
        select s.display_name, count(*), sum(d.end - d.start), max(s.arch_vgpr_count), max(s.accum_vgpr_count),
               max(d.group_segment_size)
        from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
        group by s.display_name order by sum(d.end - d.start) desc""").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"# total GPU kernel time {tot / 1e6:.3f} ms over {a.steps:g} steps = {tot / 1e6 / a.steps:.3f} ms/step")
    print("# ms_per_step   share  calls   avg_us  vgpr agpr   lds  kernel")
    for name, n, t, vg, ag, lds in rows[:a.top]:
        print(f"{t / 1e6 / a.steps:12.3f} {100 * t / tot:6.2f}% {n:6d} {t / n / 1e3:8.1f} {vg:5d} {ag:4d} {lds:5d}  "
              f"{name[:a.width]}")


if __name__ == "__main__":
    sys.exit(main())
