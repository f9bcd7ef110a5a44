"""Dispatch timeline of ONE training step from a rocprofv3 rocpd database
(``rocprofv3 --kernel-trace -d DIR -o NAME --output-format rocpd``).

The step is the span between the last two dispatches of the marker kernel
(default: the fused optimiser ``opt_k``, launched once per step).  Prints one
line per dispatch (order, us, grid, kernel) and a per-kernel-family summary,
so a layer's kernels can be located by their position and grid shape.

    python tools/step_timeline.py gpurun_out/prof12/r50_results.db > profiles/x.txt
"""
import argparse
import re
import sqlite3
import sys


def short(name: str) -> str:
    m = re.search(r"sg::(\w+)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.search(r"_ZN2sg\d+(\w+?)I", name)
    if m:
        return m.group(1)
    m = re.search(r"sg::(\w+)", name)
    if m:
        return m.group(1)
    return name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="opt_k")
    ap.add_argument("--summary-only", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("""
        select s.display_name, d.start, d.end, d.grid_size_x, d.grid_size_y, d.grid_size_z, d.workgroup_size_x
        from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
        order by d.start""").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < 2:
        print("need two marker dispatches", file=sys.stderr)
        return 1
    lo, hi = marks[-2] + 1, marks[-1] + 1
    step = rows[lo:hi]
    wall = (step[-1][2] - step[0][1]) / 1e3
    busy = sum(r[2] - r[1] for r in step) / 1e3
    print(f"# one step: {len(step)} dispatches, wall {wall:.1f} us, kernel-busy {busy:.1f} us")
    fam = {}
    for i, (name, s, e, gx, gy, gz, wx) in enumerate(step):
        k = short(name)
        f = fam.setdefault(k, [0, 0.0])
        f[0] += 1
        f[1] += (e - s) / 1e3
        if not a.summary_only:
            print(f"{i:5d} {(e - s) / 1e3:9.1f}  grid=({gx // max(1, wx)},{gy},{gz}) {k}")
    print("# per kernel family: calls, ms")
    for k, (n, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"#  {t / 1e3:8.3f} ms {n:5d}  {k}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
