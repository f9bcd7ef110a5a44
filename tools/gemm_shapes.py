"""Per-shape time of the GEMM kernels of a profiled step: joins the
``SG_GEMM_LOG=1`` launch log (igemm.hip: an ``SG_GEMM`` shape line per
``launch()`` call, an ``SG_GEMM_L`` line per kernel launched) with the GEMM
dispatches of a rocprofv3 rocpd database, in launch order.

    SG_GEMM_LOG=1 rocprofv3 --kernel-trace -d D -o x --output-format rocpd -- \\
        python3 bench.py --eager --steps 2 --warmup 1 --no-ps-parity 2> gemm.log
    python tools/gemm_shapes.py D/.../x_results.db gemm.log --steps 3

Prints one line per (kernel, shape) with calls/step, mean us, TB/s of the
compulsory bytes (A + B + C once, bf16) and TFLOP/s.
"""
import argparse
import re
import sqlite3
from collections import defaultdict

KERNELS = ("igemm_k", "pp_gemm_k", "sk_gemm_k")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("log")
    ap.add_argument("--steps", type=float, default=1.0)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("""select s.display_name, d.end - d.start from rocpd_kernel_dispatch d
                          join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.id""").fetchall()
    disp = [(n, t) for n, t in rows if any(k in n for k in KERNELS)]
    shape = None
    launches = []
    for ln in open(a.log, errors="replace"):
        if ln.startswith("SG_GEMM "):
            shape = dict(kv.split("=") for kv in ln.split()[1:])
        elif ln.startswith("SG_GEMM_L "):
            launches.append((ln.split()[1], shape))
            shape = None
    def key_of(name):
        m = re.search(r"(igemm_k|pp_gemm_k|sk_gemm_k)<([^>]*)>", name)
        return (m.group(1) + "<" + m.group(2).replace(" ", "") + ">") if m else name

    # greedy in-order alignment: a dispatch takes the next logged launch of the
    # same kernel instantiation; dispatches launched by unlogged paths are
    # counted apart
    pairs, unlogged, j = [], defaultdict(list), 0
    for name, dur in disp:
        k = key_of(name)
        if j < len(launches) and key_of(launches[j][0]) == k:
            pairs.append((launches[j], dur))
            j += 1
        else:
            unlogged[k].append(dur)
    print(f"# {len(disp)} GEMM dispatches, {len(launches)} logged launches, {len(pairs)} aligned, "
          f"{sum(len(v) for v in unlogged.values())} dispatches from unlogged paths")
    agg = defaultdict(list)
    for (kname, sh), dur in pairs:
        key = (kname,) + ((sh.get("am"), sh.get("bm"), sh.get("M"), sh.get("N"), sh.get("K"), sh.get("smode"),
                            sh.get("stats"), sh.get("res"), sh.get("beta"), sh.get("R"), sh.get("sh"))
                           if sh else ("?",) * 11)
        agg[key].append(dur)
    tot = sum(sum(v) for v in agg.values())
    print(f"# total {tot / 1e6 / a.steps:.3f} ms/step")
    print("#  ms/step calls/st  mean_us   TB/s  TF/s  kernel am bm M N K smode stats res beta R sh")
    for key, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        ms = sum(v) / 1e6 / a.steps
        us = sum(v) / len(v) / 1e3
        tb = tf = 0.0
        try:
            M, N, K = int(key[3]), int(key[4]), int(key[5])
            tb = 2.0 * (M * K + N * K + M * N) / (us * 1e-6) / 1e12
            tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        except (TypeError, ValueError):
            pass
        print(f"{ms:9.3f} {len(v) / a.steps:7.1f} {us:8.1f} {tb:6.2f} {tf:5.0f}  " + " ".join(str(k) for k in key))
    for k, v in sorted(unlogged.items(), key=lambda kv: -sum(kv[1])):
        print(f"# unlogged {sum(v) / 1e6 / a.steps:9.3f} ms/step {len(v) / a.steps:7.1f} calls/step  {k}")


if __name__ == "__main__":
    main()
