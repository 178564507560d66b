"""oracle/cpu_ref through ctypes -- the cpu_baseline leg's timer and the GPU run's checker
(test/bench infrastructure, never on the product path)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "oracle", "build", "libcpuref.so")


def pin_one_core() -> None:
    try:
        os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
    except Exception:
        pass


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return ""


class CpuRef:
    """one cpu_ref context holding host relations (column-major numpy uint64 arrays)"""

    def __init__(self):
        if not os.path.exists(SO):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "cpuref"], check=True)
        lib = C.CDLL(SO)
        lib.cpuref_create.restype = C.c_void_p
        lib.cpuref_add_relation.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p)]
        lib.cpuref_run_str.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        lib.cpuref_destroy.argtypes = [C.c_void_p]
        self.lib, self.h, self.keep = lib, lib.cpuref_create(), []

    def add_relation(self, cols) -> None:
        arr = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        self.keep.append((arr, cols))
        self.lib.cpuref_add_relation(self.h, len(cols[0]) if len(cols) else 0, len(cols), arr)

    def run(self, text: str) -> tuple[str, int, float]:
        """(stdout, rc, seconds)"""
        out, n = C.c_void_p(), C.c_size_t()
        t0 = time.perf_counter()
        rc = self.lib.cpuref_run_str(self.h, text.encode(), C.byref(out), C.byref(n))
        dt = time.perf_counter() - t0
        return C.string_at(out, n.value).decode("latin-1"), rc, dt

    def close(self) -> None:
        if self.h:
            self.lib.cpuref_destroy(self.h)
            self.h = None
        self.keep = []
