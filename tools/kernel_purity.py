"""Kernel-purity summary of a rocprofv3 kernel trace: which kernels of a
training step are this framework's own gfx950 code, and which came from
PyTorch (``at::native``), hipBLAS/hipBLASLt (``Cijk_*``), MIOpen or RCCL.

    rocprofv3 --kernel-trace -d DIR -o NAME --output-format rocpd -- python3 <workload>
    python tools/kernel_purity.py DIR/.../NAME_results.db --workload resnet50_b1024 [--json out.json]

Categories:
  native   -- singa_amd/_C kernels (namespace ``sg::``)
  copy     -- memset / memcpy / fill-with-zero and layout-free copies the runtime issues
  torch    -- PyTorch ATen compute kernels (anything else from libtorch)
  vendor   -- hipBLAS(Lt) ``Cijk_*`` / rocBLAS / MIOpen kernels
  comm     -- RCCL kernels
A step is "pure" when the torch and vendor categories are empty.
"""
from __future__ import annotations

import argparse
import json
import re
import sqlite3
import sys

_COPY = re.compile(r"(__amd_rocclr_(copy|fill)|FillFunctor<.*(0|zero)|memset|Memset|copyBuffer|fillBuffer)",
                   re.I)
_VENDOR = re.compile(r"(^Cijk_|rocblas|MIOpen|miopen|naive_conv|igemm_(fwd|bwd|wrw)_gtc|gridwise_|"
                     r"ck::|composable_kernel|hipblaslt|_Z.*Tensile)", re.I)
_COMM = re.compile(r"(nccl|rccl)", re.I)


_NATIVE = re.compile(r"(^|[\s<(,])sg::|^_ZN2sg|^_ZL\d+sg_|^sg_|(^|\s)void sg::")


def classify(name: str) -> str:
    if _NATIVE.search(name):
        return "native"
    if _COMM.search(name):
        return "comm"
    if _VENDOR.search(name):
        return "vendor"
    if _COPY.search(name):
        return "copy"
    return "torch"


def summarize(db: str, steps: float = 1.0) -> dict:
    if db.endswith(".json"):  # re-classify an earlier summary
        with open(db) as f:
            rows = [(k["kernel"], k["calls"], k["ms"] * 1e6) for k in json.load(f)["kernels"]]
    else:
        c = sqlite3.connect(db)
        rows = c.execute("""
            select s.display_name, count(*), sum(d.end - d.start)
            from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
            group by s.display_name order by sum(d.end - d.start) desc""").fetchall()
    cats: dict = {}
    kernels = []
    for name, n, t in rows:
        k = classify(name)
        e = cats.setdefault(k, {"calls": 0, "ms": 0.0})
        e["calls"] += n
        e["ms"] += t / 1e6
        kernels.append({"kernel": name[:160], "category": k, "calls": n, "ms": round(t / 1e6, 4)})
    tot = sum(e["ms"] for e in cats.values()) or 1.0
    for e in cats.values():
        e["share"] = round(e["ms"] / tot, 5)
        e["ms_per_step"] = round(e["ms"] / steps, 4)
        e["ms"] = round(e["ms"], 4)
    impure = [k for k in kernels if k["category"] in ("torch", "vendor")]
    return {"total_ms": round(tot, 4), "steps": steps, "categories": cats, "pure": not impure,
            "impure_kernels": impure, "kernels": kernels}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--workload", default="")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    s = summarize(a.db, a.steps)
    s["workload"] = a.workload
    print(f"# kernel purity: {a.workload}  total {s['total_ms']:.3f} ms  pure={s['pure']}")
    for k, e in sorted(s["categories"].items(), key=lambda kv: -kv[1]["ms"]):
        print(f"#   {k:7s} {e['ms']:10.3f} ms {100 * e['share']:6.2f}%  calls {e['calls']}")
    print("# non-native compute kernels (torch / vendor):" if s["impure_kernels"] else "# no torch / vendor kernels")
    for k in s["impure_kernels"]:
        print(f"  {k['category']:6s} {k['ms']:9.3f} ms {k['calls']:6d}x  {k['kernel']}")
    print("# all kernels:")
    for k in s["kernels"]:
        print(f"  {k['category']:6s} {k['ms']:9.3f} ms {k['calls']:6d}x  {k['kernel']}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(s, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
