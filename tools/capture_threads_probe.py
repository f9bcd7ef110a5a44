"""Probe: which cross-thread stream-capture patterns does this HIP runtime
accept?  (The loopback world captures every rank thread's step into one
graph.)  Each variant runs in order; a variant that crashes the process ends
the probe, so the variants are ordered from the most to the least likely to
work.

    python tools/capture_threads_probe.py VARIANT
      single   one thread: begin on S0, fork S1 (record E on S0, S1 waits E), kernel on S1, join, end
      launchB  thread A begins and forks; thread B launches the kernel on S1; A joins and ends
      forkB    thread A begins; thread B forks S1, launches, records the join event; A joins and ends
      tempev   one thread, the fork event destroyed right after the wait (before the capture ends)
      xrank1   the loopback world's captured all-reduce pattern between two "ranks", one thread
      xrank2   the same with each rank's calls on its own thread
      xorig1   the reduction on the ORIGIN stream instead of rank 0's comm stream (one thread)
      xorig2   the same, threaded
      multifork  the DistOpt bucket pattern: origin -> comm stream forked once per bucket (3), every
                 bucket joined back at the end
      forkjoin   fork -> kernel -> join per bucket (3), sequentially
      chain      two side streams forked from the origin, the second waiting on the first's event
      nested     a side stream forked from another side stream, both joined back to the origin
"""
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    run_variant(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)


def run_variant(variant: str, mode: int = 1):
    from singa_amd import memory, stream
    from singa_amd.ops import glue as G
    from singa_amd.ops import native as N

    rt = N.lib().rt
    dev = torch.device("cuda", 0)
    s0, s1 = stream.Stream(dev), stream.Stream(dev)
    x = memory.empty((1 << 20,), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    g = rt.Graph()
    box = {}

    def fork():
        ev = stream.Event().record(s0)
        ev.wait(s1)
        box["fork"] = ev

    def launch():
        with s1:
            G.fill_(x, 3.0)

    def join_ev():
        box["join"] = stream.Event().record(s1)

    def run_in_thread(f):
        t = threading.Thread(target=f)
        t.start()
        t.join()

    if variant.startswith("xrank"):
        return xrank(variant == "xrank2", mode)
    if variant in ("multifork", "forkjoin", "chain", "nested"):
        return patterns(variant, mode)
    if variant.startswith("xorig"):
        return xrank(variant == "xorig2", mode, on_origin=True)
    g.begin(s0.handle, mode)
    if variant == "single":
        fork(); launch(); join_ev()
    elif variant == "launchB":
        fork(); run_in_thread(launch); join_ev()
    elif variant == "forkB":
        run_in_thread(lambda: (fork(), launch(), join_ev()))
    elif variant == "tempev":
        stream.Event().record(s0).wait(s1)
        launch(); join_ev()
    box["join"].wait(s0)
    g.end()
    print(variant, "captured nodes", g.nodes, flush=True)
    G.fill_(x, 0.0)
    torch.cuda.synchronize()
    g.replay(s0.handle)
    s0.synchronize()
    v = float(G.to_numpy(x[:1])[0])
    print(variant, "replayed, x[0] =", v, flush=True)
    assert v == 3.0


def patterns(variant: str, mode: int):
    from singa_amd import memory, stream
    from singa_amd.ops import glue as G
    from singa_amd.ops import native as N

    rt = N.lib().rt
    dev = torch.device("cuda", 0)
    o = stream.Stream(dev)
    cs = stream.Stream(dev, priority=-1)
    s2 = stream.Stream(dev)
    xs = [memory.empty((4096,), dtype=torch.float32, device=dev) for _ in range(3)]
    torch.cuda.synchronize()
    g = rt.Graph()
    g.begin(o.handle, mode)
    joins = []
    if variant in ("multifork", "forkjoin"):
        for b in range(3):
            with o:
                G.fill_(xs[b], 1.0)
            cs.wait_stream(o)
            with cs:
                G.binary("mul", xs[b], 2.0, out=xs[b])
            ev = stream.Event().record(cs)
            if variant == "forkjoin":
                ev.wait(o)
            else:
                joins.append(ev)
        for ev in joins:
            ev.wait(o)
        expect = [2.0, 2.0, 2.0]
    elif variant == "chain":
        with o:
            G.fill_(xs[0], 1.0)
        cs.wait_stream(o)
        s2.wait_stream(o)
        with cs:
            G.fill_(xs[1], 3.0)
        cs_ev = stream.Event().record(cs)
        cs_ev.wait(s2)
        with s2:
            G.binary("add", xs[1], xs[0], out=xs[2])
        stream.Event().record(s2).wait(o)
        stream.Event().record(cs).wait(o)
        expect = [1.0, 3.0, 4.0]
    else:  # nested
        with o:
            G.fill_(xs[0], 1.0)
        cs.wait_stream(o)
        with cs:
            G.fill_(xs[1], 3.0)
        s2.wait_stream(cs)
        with s2:
            G.binary("add", xs[1], xs[0], out=xs[2])
        stream.Event().record(s2).wait(o)
        stream.Event().record(cs).wait(o)
        expect = [1.0, 3.0, 4.0]
    g.end()
    print(variant, "captured nodes", g.nodes, flush=True)
    for x in xs:
        G.fill_(x, 0.0)
    torch.cuda.synchronize()
    g.replay(o.handle)
    o.synchronize()
    v = [float(G.to_numpy(x[:1])[0]) for x in xs]
    print(variant, "replayed", v, flush=True)
    assert v == expect, v


def xrank(threaded: bool, mode: int, on_origin: bool = False):
    """rank r: cur_r joins the origin, cs_r forks from cur_r, records E_r;
    rank 0's cs waits every E_r and runs the reduction, records d; the other
    ranks' cs wait d; each cur_r joins its cs_r; the origin joins each cur_r."""
    from singa_amd import memory, stream
    from singa_amd.ops import glue as G
    from singa_amd.ops import native as N

    rt = N.lib().rt
    dev = torch.device("cuda", 0)
    origin = stream.Stream(dev)
    cur = [stream.Stream(dev) for _ in range(2)]
    cs = [stream.Stream(dev, priority=-1) for _ in range(2)]
    xs = [memory.empty((4096,), dtype=torch.float32, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    g = rt.Graph()
    keep = []
    bar = threading.Barrier(2 if threaded else 1)
    E = [None, None]
    box = {}

    def part1(r):
        stream.Event().record(origin).wait(cur[r])
        with cur[r]:
            G.fill_(xs[r], float(r + 1))
        cs[r].wait_stream(cur[r])
        E[r] = stream.Event().record(cs[r])

    red = origin if on_origin else cs[0]

    def part2(r):
        if r == 0:
            for j in range(2):
                if on_origin or j:
                    E[j].wait(red)
            with red:
                G.binary("add", xs[0], xs[1], out=xs[0])
                G.copy_(xs[1], xs[0])
            box["d"] = stream.Event().record(red)

    def part3(r):
        if r != 0 or on_origin:
            box["d"].wait(cs[r])
        w = stream.Event().record(cs[r])
        w.wait(cur[r])
        keep.append(stream.Event().record(cur[r]))

    g.begin(origin.handle, mode)
    if threaded:
        def body(r):
            part1(r); bar.wait(); part2(r); bar.wait(); part3(r)
        ts = [threading.Thread(target=body, args=(r,)) for r in range(2)]
        [t.start() for t in ts]
        [t.join() for t in ts]
    else:
        for f in (part1, part2, part3):
            for r in range(2):
                f(r)
    for ev in keep:
        ev.wait(origin)
    g.end()
    print("xrank captured nodes", g.nodes, flush=True)
    g.replay(origin.handle)
    origin.synchronize()
    v = [float(G.to_numpy(x[:1])[0]) for x in xs]
    print("xrank replayed", v, flush=True)
    assert v == [3.0, 3.0]


if __name__ == "__main__":
    main()
