"""Do independent kernels on two streams overlap - eagerly, and inside a captured hipGraph (fork/join
branches)?  And what does a graph launch cost?  (Decides whether scan-independent work can run beside
the persistent RSSM scan, and what cutting the step graph into pieces costs.)

    python scripts/overlap_probe.py
"""
import json
import time

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best * 1e3


def main():
    cyc = 2_000_000
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    one = timed(lambda: torch.cuda._sleep(cyc))

    def two_eager():
        ev = torch.cuda.Event()
        ev.record(main_s)
        side.wait_event(ev)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        main_s.wait_stream(side)

    eager2 = timed(two_eager)

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s0 = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(s0)
        side.wait_event(ev)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        s0.wait_stream(side)
    graph2 = timed(lambda: g.replay())

    # graph launch overhead: an empty-ish graph of 1 tiny kernel, replayed back to back
    x = torch.zeros(16, device="cuda")
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        x.add_(1)
    n = 200
    t_one = timed(lambda: [g1.replay() for _ in range(n)]) / n
    # the same kernel count as 5 graphs of 100 kernels vs 1 graph of 500
    g100 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g100):
        for _ in range(100):
            x.add_(1)
    g500 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g500):
        for _ in range(500):
            x.add_(1)
    t5x100 = timed(lambda: [g100.replay() for _ in range(5)])
    t1x500 = timed(lambda: g500.replay())
    print(json.dumps({
        "sleep_one_ms": round(one, 3), "two_streams_eager_ms": round(eager2, 3), "two_branches_graph_ms": round(graph2, 3),
        "eager_overlap": eager2 < 1.5 * one, "graph_branch_overlap": graph2 < 1.5 * one,
        "graph_replay_1kernel_us": round(t_one * 1e3, 2), "5_graphs_x_100_kernels_ms": round(t5x100, 3),
        "1_graph_x_500_kernels_ms": round(t1x500, 3),
    }))


if __name__ == "__main__":
    main()
