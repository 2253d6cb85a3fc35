"""Does a hipGraph replay run independent branches (captured on forked streams)
concurrently?  Two torch.cuda._sleep kernels on two streams: ~1x time if concurrent,
~2x if the graph serialises its branches."""
import time

import torch


def timed(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    cyc = 2_000_000
    s1 = torch.cuda.Stream()
    one = timed(lambda: torch.cuda._sleep(cyc))
    g_ser = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_ser):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
    g_par = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_par):
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cyc)
        cur.wait_stream(s1)
    # eager two streams
    def eager():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cyc)
        cur.wait_stream(s1)
    print(f"one sleep kernel eager: {one:.1f} us")
    print(f"graph, 2 serial: {timed(g_ser.replay):.1f} us")
    print(f"graph, 2 branches: {timed(g_par.replay):.1f} us")
    print(f"eager, 2 streams: {timed(eager):.1f} us")


if __name__ == "__main__":
    main()
