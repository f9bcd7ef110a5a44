"""Whole-step roofline from rocprofv3 databases: per kernel (aggregated by
name, per step) the time, HBM bytes read / written (FETCH_SIZE /
WRITE_SIZE, KB), bf16 MFMA work (SQ_INSTS_MFMA x 16384 FLOP: every bf16
kernel of the step issues v_mfma_f32_16x16x32_bf16), the achieved TB/s and
TFLOP/s, and the kernel's floor max(bytes / BW, FLOP / PEAK) with BW = the
measured device-copy bandwidth (profiles/bw_probe_copy.jsonl, 6.3 TB/s) and
PEAK = 2.5 PF dense bf16.  The step total and its floor close the table.

    python tools/step_roofline.py --steps 5 --trace trace.db pmc1.db pmc2.db pmc3.db
"""
import argparse
import sqlite3
from collections import defaultdict

BW = 6.3e12      # B/s, measured copy
PEAK = 2.5e15    # FLOP/s, dense bf16 MFMA
MFMA_FLOP = 16 * 16 * 32 * 2


def kernel_times(db):
    c = sqlite3.connect(db)
    q = """select s.display_name, count(*), sum(d_end - d_start) from (
             select kernel_id, start as d_start, end as d_end from rocpd_kernel_dispatch) k
           join rocpd_info_kernel_symbol s on k.kernel_id = s.id group by s.display_name"""
    try:
        rows = list(c.execute(q))
    except sqlite3.Error:
        rows = list(c.execute("""select s.display_name, count(*), sum(k.end - k.start)
                                 from rocpd_kernel_dispatch k join rocpd_info_kernel_symbol s
                                 on k.kernel_id = s.id group by s.display_name"""))
    return {n: (cnt, ns) for n, cnt, ns in rows}


def pmc(db):
    c = sqlite3.connect(db)
    q = """select s.display_name, i.name, sum(e.value)
           from rocpd_pmc_event e join rocpd_info_pmc i on e.pmc_id = i.id
           join rocpd_event ev on e.event_id = ev.id
           join rocpd_kernel_dispatch d on d.event_id = ev.id
           join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by s.display_name, i.name"""
    out = defaultdict(dict)
    for name, cname, v in c.execute(q):
        out[name][cname] = v
    return out


def short(n, w=64):
    n = n.replace("(sg::GemmArgs)", "").replace("void ", "")
    return n if len(n) <= w else n[:w - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, required=True, help="steps in the profiled run (warmup + timed)")
    ap.add_argument("--trace", required=True)
    ap.add_argument("pmc", nargs="+")
    a = ap.parse_args()
    t = kernel_times(a.trace)
    counters = defaultdict(dict)
    for db in a.pmc:
        for k, d in pmc(db).items():
            counters[k].update(d)
    rows = []
    for name, (cnt, ns) in t.items():
        d = counters.get(name, {})
        ms = ns / 1e6 / a.steps
        rd = d.get("FETCH_SIZE", 0.0) * 1024 / a.steps
        wr = d.get("WRITE_SIZE", 0.0) * 1024 / a.steps
        fl = d.get("SQ_INSTS_MFMA", 0.0) * MFMA_FLOP / a.steps
        floor = max((rd + wr) / BW, fl / PEAK) * 1e3
        rows.append((ms, rd, wr, fl, floor, cnt / a.steps, name))
    rows.sort(key=lambda r: -r[0])
    T = sum(r[0] for r in rows)
    R = sum(r[1] for r in rows)
    W = sum(r[2] for r in rows)
    Fl = sum(r[3] for r in rows)
    Fk = sum(r[4] for r in rows)
    print(f"# whole-step roofline, per step (BW {BW / 1e12:.1f} TB/s copy, PEAK {PEAK / 1e15:.1f} PF bf16)")
    print(f"# {'ms':>7} {'GB rd':>7} {'GB wr':>7} {'TB/s':>6} {'TFLOP':>7} {'TF/s':>7} {'floor':>7} {'%flr':>5} "
          f"{'calls':>6}  kernel")
    for ms, rd, wr, fl, floor, cnt, name in rows:
        if ms < 0.02:
            continue
        print(f"  {ms:7.3f} {rd / 1e9:7.2f} {wr / 1e9:7.2f} {(rd + wr) / ms / 1e9:6.2f} {fl / 1e12:7.2f} "
              f"{fl / ms / 1e9:7.1f} {floor:7.3f} {100 * floor / ms:5.1f} {cnt:6.1f}  {short(name)}")
    print(f"# step: {T:.2f} ms kernel time, {R / 1e9:.1f} GB read + {W / 1e9:.1f} GB written, {Fl / 1e12:.1f} TFLOP")
    print(f"# memory floor {(R + W) / BW * 1e3:.2f} ms, compute floor {Fl / PEAK * 1e3:.2f} ms, "
          f"sum of per-kernel floors {Fk:.2f} ms -> the step runs at {100 * Fk / T:.1f} % of its per-kernel floor")


if __name__ == "__main__":
    main()
