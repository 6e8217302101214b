"""Do independent branches of a captured HIP graph run concurrently?
Two streams, each a chain of small latency-bound kernels (elementwise ops on
small tensors), captured fork/join; compare replay time with the serial
capture of the same kernels."""
import torch

dev = "cuda"
n_k = 200
a = torch.randn(1 << 16, device=dev)
b = torch.randn(1 << 16, device=dev)
s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()


def chain(t):
    for _ in range(n_k):
        t.mul_(1.0001).add_(1e-4)


def serial():
    chain(a)
    chain(b)


def forked():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        chain(a)
    with torch.cuda.stream(s2):
        chain(b)
    cur.wait_stream(s1)
    cur.wait_stream(s2)


def timeit(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[2] * 1e3


ts = timeit(serial)
tf = timeit(forked)
print("serial %.1f us (%.2f us/kernel), forked %.1f us -> ratio %.2f" % (ts, ts / (4 * n_k), tf, tf / ts))
