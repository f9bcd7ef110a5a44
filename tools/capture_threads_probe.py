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
"""
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from singa_amd import memory, stream
    from singa_amd.ops import glue as G
    from singa_amd.ops import native as N

    variant = sys.argv[1]
    mode = int(sys.argv[2]) if len(sys.argv) > 2 else 2
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


if __name__ == "__main__":
    main()
