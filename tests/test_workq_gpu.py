"""Dynamic work queues of the persistent kernels (csrc/kernels/workq.hip,
common.h): sk_gemm_k (1x1-conv GEMMs), conv3x3_k (stage-1 3x3) and
stem_fwd_k take their units from a device counter that the last workgroup
resets.  Checked here:

* queue on == static partition, bit for bit (the queue only reorders work);
* back-to-back launches and graph replays reuse a slot correctly (the
  output buffer is NaN-filled before every launch, so a slot that was not
  reset -- tickets starting past the end -- would leave NaN tiles);
* with 32 CUs held by a concurrent "CU hog" on another stream (a stand-in for
  RCCL's channel kernels) the results are unchanged.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cases(L, dev):
    """name -> (launch on the current stream, output buffer)"""
    from singa_amd.ops import native as N

    n = 128
    g = torch.Generator(device=dev).manual_seed(5)
    out = {}
    for (h, c, k) in ((56, 64, 256), (28, 128, 512)):
        x = torch.randn(n, h, h, c, device=dev, generator=g).bfloat16()
        w = (torch.randn(k, 1, 1, c, device=dev, generator=g) * 0.1).bfloat16()
        y = torch.empty(n, h, h, k, device=dev, dtype=torch.bfloat16)

        def f(x=x, w=w, y=y, h=h, c=c, k=k):
            L.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, n, h, h, c, k, 1, 1, h, h, 1, 1, 0, 0, 1, 1, 0, 0,
                       N.stream(), 0)
        out[f"sk_{h}_{c}x{k}"] = (f, y)
    x = torch.randn(n, 56, 56, 64, device=dev, generator=g).bfloat16()
    w = (torch.randn(64, 3, 3, 64, device=dev, generator=g) * 0.05).bfloat16()
    y3 = torch.empty_like(x)

    def c3():
        L.conv_fwd(x.data_ptr(), w.data_ptr(), y3.data_ptr(), 0, n, 56, 56, 64, 64, 3, 3, 56, 56, 1, 1, 1, 1, 1, 1, 0,
                   0, N.stream(), 0)
    out["conv3x3"] = (c3, y3)
    xp = torch.randn(16, 224, 225, 8, device=dev, generator=g).bfloat16()
    wp = (torch.randn(64, 224, device=dev, generator=g) * 0.05).bfloat16()
    ys = torch.empty(16, 112, 112, 64, device=dev, dtype=torch.bfloat16)

    def stem():
        assert L.stem_fwd(xp.data_ptr(), wp.data_ptr(), ys.data_ptr(), 0, 16, 224, 225, 112, 112, N.stream())
    out["stem"] = (stem, ys)
    return out


@pytest.fixture
def lib(gpu):
    from singa_amd.ops import native as N

    L = N.lib()
    yield L
    L.workq_set(1)


def test_queue_matches_static_and_resets(gpu, lib):
    L = lib
    for name, (fn, y) in _cases(L, gpu).items():
        L.workq_set(0)
        y.fill_(float("nan"))
        fn()
        ref = y.clone()
        assert not torch.isnan(ref).any(), name
        L.workq_set(1)
        for rep in range(4):  # back-to-back launches reuse ring slots after their reset
            y.fill_(float("nan"))
            fn()
            torch.cuda.synchronize()
            assert torch.equal(y, ref), (name, rep)


def test_queue_under_cu_hog(gpu, lib):
    from singa_amd.ops import native as N

    L = lib
    L.workq_set(1)
    s = N.stream()
    side = torch.cuda.Stream()
    started = torch.zeros(1, dtype=torch.int32, device=gpu)
    for name, (fn, y) in _cases(L, gpu).items():
        fn()
        ref = y.clone()
        y.fill_(float("nan"))
        torch.cuda.synchronize()
        L.cu_hog(32, 20000.0, 0, started.data_ptr(), side.cuda_stream)
        L.cu_hog(1, 50.0, 0, 0, s)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        assert torch.equal(y, ref), name
    assert int(started.item()) == 32 * 4


def test_queue_graph_replay(gpu, lib):
    """A captured launch keeps its queue slot; the device-side reset makes every
    replay start from zero."""
    from singa_amd.stream import StepGraph

    L = lib
    L.workq_set(1)
    cases = _cases(L, gpu)
    refs = {}
    for name, (fn, y) in cases.items():
        fn()
        refs[name] = y.clone()
    torch.cuda.synchronize()

    def step():
        for fn, _ in cases.values():
            fn()

    g = StepGraph()
    g.capture(step)
    for rep in range(3):
        for _, (_, y) in cases.items():
            y.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        for name, (_, y) in cases.items():
            assert torch.equal(y, refs[name]), (name, rep)
    g.release()


def test_two_graphs_replayed_concurrently_own_their_slots(gpu, lib):
    """Two graphs capturing the same persistent kernels, replayed at the same
    time on two streams while eager launches of those kernels run on a third:
    each capture takes its queue slots from its own arena (never from the
    shared ring the eager launches advance), so no two running kernels share
    counters and every output is exact."""
    from singa_amd import stream as S
    from singa_amd.stream import StepGraph

    L = lib
    L.workq_set(1)
    sets = [_cases(L, gpu) for _ in range(3)]
    refs = []
    for cases in sets:
        r = {}
        for name, (fn, y) in cases.items():
            fn()
            r[name] = y.clone()
        refs.append(r)
    torch.cuda.synchronize()
    graphs = []
    for cases in sets[:2]:
        g = StepGraph()
        g.capture(lambda cases=cases: [fn() for fn, _ in cases.values()])
        assert g.queue_slots == len(cases), g.queue_slots  # one fresh slot per captured persistent launch
        graphs.append(g)
    streams = [S.pooled(gpu, f"wq-test-{i}") for i in range(3)]
    for rep in range(4):
        for cases in sets:
            for _, y in cases.values():
                y.fill_(float("nan"))
        torch.cuda.synchronize()
        for g, s in zip(graphs, streams[:2]):
            with s:
                g.replay()
        with streams[2]:
            for _ in range(2):
                for fn, _ in sets[2].values():
                    fn()
        torch.cuda.synchronize()
        for cases, r in zip(sets, refs):
            for name, (_, y) in cases.items():
                assert torch.equal(y, r[name]), (name, rep)
    for g in graphs:
        g.release()


def test_queue_stress_back_to_back(gpu, lib):
    """Many back-to-back launches of each persistent kernel, the output
    NaN-filled before every launch and checked on the device (no host sync
    in between, so kernel ends and the next launch's first tickets overlap as
    in a training step): a ticket that lands after the last workgroup's reset
    would skip a work unit of a later launch on that slot and leave NaN."""
    L = lib
    L.workq_set(1)
    cases = _cases(L, gpu)
    bad = torch.zeros(len(cases), dtype=torch.int32, device=gpu)
    for ci, (name, (fn, y)) in enumerate(cases.items()):
        fn()
        ref = y.clone()
        for _ in range(60):
            y.fill_(float("nan"))
            fn()
            bad[ci] += (~torch.eq(y, ref)).any().int()
    torch.cuda.synchronize()
    assert bad.tolist() == [0] * len(cases), dict(zip(cases, bad.tolist()))
