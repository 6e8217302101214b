"""Per-kernel time of graph-replayed kernels with K dependent global loads
(each kernel reads what the previous one wrote): the marginal cost of one
memory round trip inside a launch, at several grid sizes and working sets."""
import ctypes as C
import os

lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liblatency_chain.so"))
lib.probe_chain.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double)]
for grid in (256, 1024, 4096):
    for n in (1 << 16, 1 << 20, 1 << 24):
        us = (C.c_double * 5)()
        assert lib.probe_chain(grid, n, us) == 0
        print("grid %5d  working set %6d KB: us/kernel K=0 %.2f  K=1 %.2f  K=2 %.2f  K=4 %.2f  K=8 %.2f"
              % (grid, 4 * n // 1024, *us), flush=True)
