"""Per-kernel PMC counter sums from rocprofv3 databases (``--pmc``).
    python tools/pmc_summary.py gpurun_out/pmc1/c_results.db [more.db ...]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(int)
    for f in sys.argv[1:]:
        c = sqlite3.connect(f)
        q = """select s.display_name, d.id, i.name, sum(e.value)
               from rocpd_pmc_event e join rocpd_info_pmc i on e.pmc_id = i.id
               join rocpd_event ev on e.event_id = ev.id
               join rocpd_kernel_dispatch d on d.event_id = ev.id
               join rocpd_info_kernel_symbol s on d.kernel_id = s.id
               group by d.id, i.name"""
        seen = set()
        for name, did, cname, v in c.execute(q):
            agg[name][cname] += v
            if (f, did) not in seen:
                seen.add((f, did))
                calls[(name, f)] += 1
    for name, d in agg.items():
        print(name[:100])
        for k in sorted(d):
            print(f"   {k:32s} {d[k]:.4g}")


if __name__ == "__main__":
    main()
