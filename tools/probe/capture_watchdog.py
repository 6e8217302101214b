"""Probe (GPU box, world size 1 RCCL): does a process-group watchdog that still
holds an eager collective abort the process when a HIP graph capture is open?

    python3 tools/probe/capture_watchdog.py drained
    python3 tools/probe/capture_watchdog.py pending   # run LAST in a GPU call

Result (round 5, profiles/r5_capture_watchdog.txt): BOTH pass.  The c10d
flight recorder is off by default here (0 entries), so "drained" waits for
nothing, and "pending" -- a finished all-reduce still on the WORLD watchdog's
list while a 0.6 s thread-local capture is open -- does not abort: the
watchdog's event poll during a capture is not the round-4 abort's cause.

Both modes: one eager all_reduce on WORLD, torch.cuda.synchronize(), then a
thread-local capture of a few kernels on a side stream that stays open for
0.6 s (the c10d watchdog wakes every ~100 ms and polls the completion event of
every work it has not retired yet).  "drained" first waits until the flight
recorder reports no active (unretired) collective; "pending" captures right
after the device sync, which is what the round-4 capture() did after its
warm-up all-reduces.
"""
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
from torch._C._distributed_c10d import _dump_nccl_trace_json


def active_entries():
    d = json.loads(_dump_nccl_trace_json(True, True))
    return d.get("entries", [])


def main():
    mode = sys.argv[1]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    x = torch.ones(1 << 20, device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    all_e = json.loads(_dump_nccl_trace_json(True, False)).get("entries", [])
    print("flight recorder entries after sync: %d; active: %d" % (len(all_e), len(active_entries())), flush=True)
    for e in all_e[-2:]:
        print("  ", {k: e.get(k) for k in ("profiling_name", "state", "retired", "pg_id")}, flush=True)
    if mode == "drained":
        t0 = time.time()
        while active_entries():
            time.sleep(0.005)
        print("drained after %.3f s" % (time.time() - t0), flush=True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    y = torch.zeros_like(x)
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
            for _ in range(4):
                y.add_(x)
            time.sleep(0.6)          # capture open across several watchdog periods
    g.replay()
    torch.cuda.synchronize()
    print("capture %s ok, y[0] = %g" % (mode, float(y[0])), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
