"""ctypes binding of libqe (include/qe.h).

The product path is native: every call goes into build/libqe.so (HIP kernels for gfx950 + the
host-C executor).  There is no Python or CPU fallback -- if the library is missing or no GPU
is usable, these calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("QE_LIB_PATH") or os.path.join(PKG, "build", "libqe.so")   # override: ablation builds (tools/)
HEADER = os.path.join(os.path.dirname(PKG), "include", "qe.h")

QE_EINVAL, QE_EHIP, QE_ENOMEM, QE_EEXIT, QE_ETOOBIG, QE_ENOTSUP = -1, -2, -3, -4, -5, -6
LIST_DISTINCT = 1
PAIRS_DISTINCT, PAIRS_SORTED = 1, 2


class Col(C.Structure):
    _fields_ = [("d", C.c_void_p), ("n", C.c_uint64)]


class List(C.Structure):
    _fields_ = [("d", C.c_void_p), ("n", C.c_uint64), ("cap", C.c_uint64), ("flags", C.c_uint32)]


class Pairs(C.Structure):
    _fields_ = [("key", C.c_void_p), ("val", C.c_void_p), ("match", C.c_void_p), ("n", C.c_uint64),
                ("kor", C.c_uint64), ("kand", C.c_uint64), ("flags", C.c_uint32), ("owns", C.c_uint32)]


class KStat(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("launches", C.c_uint64), ("total_ms", C.c_double),
                ("alg_bytes", C.c_double)]


class QEError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libqe error {code}: {msg}")
        self.code = code


_lib = None


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load libqe.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: build it with __graft_entry__.build() or "
                                f"`make -C query-compiler-executor_amd` (libqe has no CPU fallback)")
    lib = C.CDLL(path)
    P, U64, I, VP = C.c_void_p, C.c_uint64, C.c_int, C.c_void_p
    sig = {
        "qe_init": (P, [I]),
        "qe_fini": (None, [P]),
        "qe_last_error": (C.c_char_p, [P]),
        "qe_abi_version": (I, []),
        "qe_device_name": (I, [P, C.c_char_p, C.c_size_t]),
        "qe_sync": (I, [P]),
        "qe_load_relation": (I, [P, U64, U64, C.POINTER(C.c_void_p)]),
        "qe_gen_relation": (I, [P, U64, U64, C.POINTER(C.c_int), C.POINTER(C.c_uint64), U64, C.c_uint32, U64]),
        "qe_relation_count": (I, [P]),
        "qe_relation_column": (I, [P, I, I, C.POINTER(Col)]),
        "qe_relation_rows": (I, [P, I, C.POINTER(C.c_uint64)]),
        "qe_drop_relations": (I, [P]),
        "qe_run_queries": (I, [P, C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
        "qe_free_host": (None, [VP]),
        "qe_last_result_rows": (I, [P, C.POINTER(C.c_uint64)]),
        "qe_set_last_result_rows": (I, [P, U64]),
        "qe_filter_scan": (I, [P, Col, C.c_char, U64, C.POINTER(List)]),
        "qe_filter_refine": (I, [P, Col, C.c_char, U64, C.POINTER(List)]),
        "qe_gather_pairs": (I, [P, Col, C.POINTER(List), C.POINTER(Pairs)]),
        "qe_sort_pairs": (I, [P, C.POINTER(Pairs)]),
        "qe_is_sorted": (I, [P, C.POINTER(Pairs), C.POINTER(C.c_int)]),
        "qe_merge_join": (I, [P, C.POINTER(Pairs), C.POINTER(Pairs), C.POINTER(List), C.POINTER(List)]),
        "qe_join_pairs": (I, [P, C.POINTER(Pairs), C.POINTER(Pairs), C.POINTER(List), C.POINTER(List)]),
        "qe_scan_join": (I, [P, C.POINTER(Pairs), C.POINTER(Pairs), C.POINTER(List), C.POINTER(List)]),
        "qe_driver_counts": (I, [P, C.POINTER(Pairs), C.POINTER(Pairs), C.POINTER(List), C.POINTER(List), I, U64,
                                 C.POINTER(C.c_void_p)]),
        "qe_join_payloads": (I, [P, C.c_void_p, U64, C.POINTER(List), C.POINTER(List), C.POINTER(List)]),
        "qe_join_payloads_multi": (I, [P, C.c_void_p, U64, C.POINTER(List), C.POINTER(C.POINTER(List)), I,
                                       C.POINTER(List)]),
        "qe_relation_column_bits": (I, [P, I, I, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "qe_checksum": (I, [P, Col, C.POINTER(List), C.POINTER(C.c_uint64)]),
        "qe_checksums": (I, [P, I, C.POINTER(Col), C.POINTER(C.POINTER(List)), C.POINTER(C.c_uint64)]),
        "qe_checksum_weighted": (I, [P, Col, C.POINTER(Pairs), C.POINTER(C.c_uint64)]),
        "qe_merge_join_counts": (I, [P, C.POINTER(Pairs), C.POINTER(Pairs), C.POINTER(C.c_uint64)]),
        "qe_join_aggregate": (I, [P, Col, Col, Col, Col, C.POINTER(C.c_uint64)]),
        "qe_set_materialize_limit": (I, [P, U64]),
        "qe_set_zipf_table": (I, [P, C.c_void_p, U64, U64]),
        "qe_set_zipf": (I, [P, U64, C.c_double, U64]),
        "qe_partition": (I, [P, C.c_void_p, U64, C.POINTER(C.c_void_p), I, C.c_uint32, C.POINTER(C.c_uint64),
                             C.c_void_p, C.POINTER(C.c_void_p)]),
        "qe_filter_scan_range": (I, [P, Col, U64, U64, C.c_char, U64, C.POINTER(List)]),
        "qe_filter_scan2_range": (I, [P, Col, C.c_char, U64, Col, C.c_char, U64, U64, U64, C.POINTER(List)]),
        "qe_iota": (I, [P, U64, U64, C.POINTER(List)]),
        "qe_take_u32": (I, [P, C.c_void_p, C.POINTER(List), C.POINTER(List)]),
        "qe_join_indices": (I, [P, C.c_void_p, U64, C.c_void_p, U64, C.POINTER(List), C.POINTER(List)]),
        "qe_sync_stream_ptr": (I, [P, C.POINTER(C.c_void_p)]),
        "qe_bucket_select": (I, [P, Col, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.POINTER(Pairs)]),
        "qe_heavy_stats": (I, [P, Col, U64, U64, C.c_void_p, C.c_uint32, Col, C.c_void_p, C.c_void_p,
                               C.POINTER(C.c_uint64)]),
        "qe_list_alloc": (I, [P, U64, C.POINTER(List)]),
        "qe_list_from_host": (I, [P, VP, U64, C.c_uint32, C.POINTER(List)]),
        "qe_list_to_host": (I, [P, C.POINTER(List), VP]),
        "qe_list_free": (None, [P, C.POINTER(List)]),
        "qe_pairs_from_host": (I, [P, VP, VP, U64, C.POINTER(Pairs)]),
        "qe_pairs_to_host": (I, [P, C.POINTER(Pairs), VP, VP]),
        "qe_pairs_free": (None, [P, C.POINTER(Pairs)]),
        "qe_counts_free": (None, [P, C.c_void_p]),
        "qe_counts_to_host": (I, [P, C.c_void_p, U64, VP]),
        "qe_mem_stats": (I, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "qe_load_stats": (I, [P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
        "qe_partition_columns": (I, [P, C.c_uint32, C.c_uint32]),
        "qe_mem_trim": (I, [P]),
        "qe_set_profiling": (I, [P, I]),
        "qe_set_profiling_only": (I, [P, C.c_char_p]),
        "qe_reset_stats": (I, [P]),
        "qe_kernel_stats": (I, [P, C.POINTER(KStat), I]),
        "qe_comm_unique_id": (I, [C.c_char_p]),
        "qe_comm_init": (I, [P, I, I, C.c_char_p, C.POINTER(C.c_void_p)]),
        "qe_comm_fini": (None, [P]),
        "qe_allreduce_u64": (I, [P, P, C.POINTER(C.c_uint64), I]),
        "qe_shuffle_pairs": (I, [P, P, C.c_void_p, U64, C.POINTER(C.c_void_p), I, C.POINTER(C.c_void_p),
                                 C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
        "qe_buffer_free": (None, [P, C.c_void_p]),
        "qe_comm_stats": (I, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "qe_run_queries_dist": (I, [P, P, C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                    C.POINTER(C.c_uint64)]),
        "qe_run_queries_parallel": (I, [P, I, C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
        "qe_run_queries_lanes": (I, [P, I, I, C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
        "qe_sort_cache": (I, [P, I]),
        "qe_sort_cache_stats": (I, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "qe_comm_init_local": (I, [C.POINTER(C.c_void_p), I, C.POINTER(C.c_void_p)]),
        "qe_run_queries_local": (I, [P, I, C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "qe_workers": (I, [P, I, C.POINTER(C.c_void_p)]),
        "qe_bind_thread": (I, [P]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("QE_LIB_PATH") and not hasattr(lib, name):
            continue   # an older ablation build (QE_LIB_PATH, tools/) may predate an entry point
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def declared_symbols(header: str = HEADER) -> list[str]:
    """Every function name include/qe.h declares."""
    import re
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(qe_[a-z0-9_]+)\s*\(", txt)))


class Ctx:
    """One device context (one HIP stream, one caching allocator)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        self.h = self.lib.qe_init(device)
        if not self.h:
            raise QEError(QE_EHIP, f"qe_init({device}) failed: no usable GPU (libqe has no CPU path)")
        self.device = device

    def close(self):
        if self.h:
            self.lib.qe_fini(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc):
        if rc < 0:
            raise QEError(rc, self.lib.qe_last_error(self.h).decode())
        return rc

    def device_name(self) -> str:
        b = C.create_string_buffer(256)
        self._chk(self.lib.qe_device_name(self.h, b, 256))
        return b.value.decode()

    # ---- relations ----
    def load_relation(self, cols: list[np.ndarray]) -> int:
        cols = [np.ascontiguousarray(c, dtype=np.uint64) for c in cols]
        rows = len(cols[0]) if cols else 0
        arr = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
        return self._chk(self.lib.qe_load_relation(self.h, rows, len(cols), arr))

    def gen_relation(self, rows: int, kinds: list[tuple], seed: int, gen_rel: int, row_start: int = 0) -> int:
        """kinds as qe.datagen: ("mod", M), ("hi32",), ("zipf", D, theta, perm_seed) -- the last
        needs set_zipf_table(cdf of (D, theta), D, perm_seed) first"""
        code = {"mod": 0, "hi32": 1, "zipf": 2}
        k = (C.c_int * len(kinds))(*[code[kd[0]] for kd in kinds])
        m = (C.c_uint64 * len(kinds))(*[int(kd[1]) if kd[0] in ("mod", "zipf") else 0 for kd in kinds])
        return self._chk(self.lib.qe_gen_relation(self.h, rows, len(kinds), k, m, seed, gen_rel, row_start))

    def set_zipf_table(self, d_cdf_ptr: int, domain: int, perm_seed: int) -> None:
        """d_cdf_ptr: device address of `domain` float64 CDF values (kept alive by the caller)"""
        self._chk(self.lib.qe_set_zipf_table(self.h, d_cdf_ptr, domain, perm_seed))

    def set_zipf(self, domain: int, theta: float, perm_seed: int) -> None:
        """Zipf table built (deterministically) and owned by libqe"""
        self._chk(self.lib.qe_set_zipf(self.h, domain, theta, perm_seed))

    def drop_relations(self):
        self._chk(self.lib.qe_drop_relations(self.h))

    def column(self, rel: int, col: int) -> Col:
        c = Col()
        self._chk(self.lib.qe_relation_column(self.h, rel, col, C.byref(c)))
        return c

    # ---- executor ----
    def run(self, text: str) -> tuple[str, int]:
        out = C.c_void_p()
        n = C.c_size_t()
        rc = self.lib.qe_run_queries(self.h, text.encode(), C.byref(out), C.byref(n))
        s = C.string_at(out, n.value).decode("latin-1") if out.value else ""
        if out.value:
            self.lib.qe_free_host(out)
        if rc not in (0, QE_EEXIT):
            raise QEError(rc, self.lib.qe_last_error(self.h).decode())
        return s, (1 if rc == QE_EEXIT else 0)

    def run_parallel(self, text: str, workers: int = 4) -> tuple[str, int]:
        """qe_run_queries_parallel: the batch's queries on `workers` concurrent lanes, same bytes"""
        out, n = C.c_void_p(), C.c_size_t()
        rc = self.lib.qe_run_queries_parallel(self.h, workers, text.encode(), C.byref(out), C.byref(n))
        s = C.string_at(out, n.value).decode("latin-1") if out.value else ""
        if out.value:
            self.lib.qe_free_host(out)
        if rc not in (0, QE_EEXIT):
            raise QEError(rc, self.lib.qe_last_error(self.h).decode())
        return s, (1 if rc == QE_EEXIT else 0)

    def run_lanes(self, text: str, workers: int = 4, plan: bool = True) -> tuple[str, int]:
        """qe_run_queries_lanes: the batch on `workers` lanes, each query through the partitioned
        plan (faithful fallback) or the faithful executor -- the same bytes either way"""
        out, n = C.c_void_p(), C.c_size_t()
        rc = self.lib.qe_run_queries_lanes(self.h, workers, 1 if plan else 0, text.encode(), C.byref(out), C.byref(n))
        s = C.string_at(out, n.value).decode("latin-1") if out.value else ""
        if out.value:
            self.lib.qe_free_host(out)
        if rc not in (0, QE_EEXIT):
            raise QEError(rc, self.lib.qe_last_error(self.h).decode())
        return s, (1 if rc == QE_EEXIT else 0)

    def sort_cache_stats(self) -> tuple[int, int]:
        """(cached base-column sorts reused, built) over this ctx's finished batches"""
        if not hasattr(self.lib, "qe_sort_cache_stats"):   # (an older ablation build)
            return 0, 0
        h, b = C.c_uint64(), C.c_uint64()
        self.lib.qe_sort_cache_stats(self.h, C.byref(h), C.byref(b))
        return h.value, b.value

    def run_dist(self, text: str, comm: "Comm | None" = None) -> tuple[str, int, int]:
        """qe_run_queries_dist: (stdout on rank 0, exit status, queries run the faithful way)"""
        out, n, ref = C.c_void_p(), C.c_size_t(), C.c_uint64()
        rc = self.lib.qe_run_queries_dist(self.h, comm.h if comm else None, text.encode(), C.byref(out), C.byref(n),
                                          C.byref(ref))
        s = C.string_at(out, n.value).decode("latin-1") if out.value else ""
        if out.value:
            self.lib.qe_free_host(out)
        if rc not in (0, QE_EEXIT):
            raise QEError(rc, self.lib.qe_last_error(self.h).decode())
        return s, (1 if rc == QE_EEXIT else 0), ref.value

    def run_local(self, text: str, nranks: int) -> tuple[str, int, int, int]:
        """qe_run_queries_local: the partitioned executor on `nranks` in-process ranks of this GPU
        (worker contexts, one host thread each) -> (stdout, exit status, refused, bytes exchanged)"""
        out, n, ref, sent = C.c_void_p(), C.c_size_t(), C.c_uint64(), C.c_uint64()
        rc = self.lib.qe_run_queries_local(self.h, nranks, text.encode(), C.byref(out), C.byref(n), C.byref(ref),
                                           C.byref(sent))
        s = C.string_at(out, n.value).decode("latin-1") if out.value else ""
        if out.value:
            self.lib.qe_free_host(out)
        if rc not in (0, QE_EEXIT):
            raise QEError(rc, self.lib.qe_last_error(self.h).decode())
        return s, (1 if rc == QE_EEXIT else 0), ref.value, sent.value

    def workers(self, n: int) -> list["Ctx"]:
        """qe_workers: n contexts on this GPU sharing its relations (owned by this ctx)"""
        arr = (C.c_void_p * n)()
        self._chk(self.lib.qe_workers(self.h, n, arr))
        out = []
        for i in range(n):
            w = Ctx.__new__(Ctx)
            w.lib, w.h, w.device = self.lib, arr[i], self.device
            w.close = lambda: None              # freed by the owning ctx's qe_fini
            out.append(w)
        return out

    def buffer_free(self, ptr: int) -> None:
        self.lib.qe_buffer_free(self.h, ptr)

    def last_result_rows(self) -> int:
        r = C.c_uint64()
        self._chk(self.lib.qe_last_result_rows(self.h, C.byref(r)))
        return r.value

    # ---- primitives (tests / bench) ----
    def list_from_host(self, a: np.ndarray, flags: int = 0) -> List:
        a = np.ascontiguousarray(a, dtype=np.uint32)
        l = List()
        self._chk(self.lib.qe_list_from_host(self.h, a.ctypes.data, len(a), flags, C.byref(l)))
        return l

    def list_to_host(self, l: List) -> np.ndarray:
        a = np.empty(l.n, dtype=np.uint32)
        self._chk(self.lib.qe_list_to_host(self.h, C.byref(l), a.ctypes.data))
        return a

    def list_free(self, l: List):
        self.lib.qe_list_free(self.h, C.byref(l))

    def pairs_from_host(self, key: np.ndarray, val: np.ndarray) -> Pairs:
        key = np.ascontiguousarray(key, dtype=np.uint64)
        val = np.ascontiguousarray(val, dtype=np.uint32)
        p = Pairs()
        self._chk(self.lib.qe_pairs_from_host(self.h, key.ctypes.data, val.ctypes.data, len(key), C.byref(p)))
        return p

    def pairs_to_host(self, p: Pairs) -> tuple[np.ndarray, np.ndarray]:
        k = np.empty(p.n, dtype=np.uint64)
        v = np.empty(p.n, dtype=np.uint32)
        self._chk(self.lib.qe_pairs_to_host(self.h, C.byref(p), k.ctypes.data, v.ctypes.data))
        return k, v

    def pairs_free(self, p: Pairs):
        self.lib.qe_pairs_free(self.h, C.byref(p))

    def filter_scan(self, col: Col, op: str, v: int) -> List:
        l = List()
        self._chk(self.lib.qe_filter_scan(self.h, col, op.encode(), v, C.byref(l)))
        return l

    def filter_refine(self, col: Col, op: str, v: int, l: List) -> List:
        self._chk(self.lib.qe_filter_refine(self.h, col, op.encode(), v, C.byref(l)))
        return l

    def gather_pairs(self, col: Col, rows: List | None) -> Pairs:
        p = Pairs()
        self._chk(self.lib.qe_gather_pairs(self.h, col, C.byref(rows) if rows is not None else None, C.byref(p)))
        return p

    def sort_pairs(self, p: Pairs) -> Pairs:
        self._chk(self.lib.qe_sort_pairs(self.h, C.byref(p)))
        return p

    def is_sorted(self, p: Pairs) -> bool:
        s = C.c_int()
        self._chk(self.lib.qe_is_sorted(self.h, C.byref(p), C.byref(s)))
        return bool(s.value)

    def merge_join(self, R: Pairs, S: Pairs) -> tuple[List, List]:
        a, b = List(), List()
        self._chk(self.lib.qe_merge_join(self.h, C.byref(R), C.byref(S), C.byref(a), C.byref(b)))
        return a, b

    def join_pairs(self, R: Pairs, S: Pairs) -> tuple[List, List]:
        """qe_join_pairs: every matching (R val, S val), aligned, in no particular order"""
        a, b = List(), List()
        self._chk(self.lib.qe_join_pairs(self.h, C.byref(R), C.byref(S), C.byref(a), C.byref(b)))
        return a, b

    def scan_join(self, R: Pairs, S: Pairs) -> tuple[List, List]:
        a, b = List(), List()
        self._chk(self.lib.qe_scan_join(self.h, C.byref(R), C.byref(S), C.byref(a), C.byref(b)))
        return a, b

    def driver_counts(self, R: Pairs | None, S: Pairs | None, outR: List, outS: List, mode: int, rows: int):
        d = C.c_void_p()
        self._chk(self.lib.qe_driver_counts(self.h, C.byref(R) if R is not None else None,
                                            C.byref(S) if S is not None else None, C.byref(outR), C.byref(outS),
                                            mode, rows, C.byref(d)))
        return d

    def counts_to_host(self, d, n: int) -> np.ndarray:
        a = np.empty(n, dtype=np.uint32)
        self._chk(self.lib.qe_counts_to_host(self.h, d, n, a.ctypes.data))
        return a

    def counts_free(self, d):
        self.lib.qe_counts_free(self.h, d)

    def join_payloads(self, counts, rows: int, last: List, edit: List) -> List:
        out = List()
        self._chk(self.lib.qe_join_payloads(self.h, counts, rows, C.byref(last), C.byref(edit), C.byref(out)))
        return out

    def join_payloads_multi(self, counts, rows: int, last: List, edits: list[List]) -> list[List]:
        arr = (C.POINTER(List) * len(edits))(*[C.pointer(e) for e in edits])
        outs = (List * len(edits))()
        self._chk(self.lib.qe_join_payloads_multi(self.h, counts, rows, C.byref(last), arr, len(edits), outs))
        return list(outs)

    def column_bits(self, rel: int, col: int) -> tuple[int, int]:
        a, b = C.c_uint64(), C.c_uint64()
        self._chk(self.lib.qe_relation_column_bits(self.h, rel, col, C.byref(a), C.byref(b)))
        return a.value, b.value

    def column_to_host(self, rel: int, col: int) -> np.ndarray:
        k = np.empty(self.column(rel, col).n, dtype=np.uint64)
        p = self.gather_pairs(self.column(rel, col), None)
        self._chk(self.lib.qe_pairs_to_host(self.h, C.byref(p), k.ctypes.data, None))
        return k

    def column_range_to_host(self, rel: int, col: int, start: int, n: int) -> np.ndarray:
        """values [start, start + n) of a device column, on the host"""
        c = self.column(rel, col)
        n = max(0, min(n, c.n - start))
        k = np.empty(n, dtype=np.uint64)
        if n:
            p = Pairs()
            p.key, p.val, p.match, p.n = c.d + 8 * start, None, None, n
            self._chk(self.lib.qe_pairs_to_host(self.h, C.byref(p), k.ctypes.data, None))
        return k

    def merge_join_counts(self, R: Pairs, S: Pairs) -> int:
        P = C.c_uint64()
        self._chk(self.lib.qe_merge_join_counts(self.h, C.byref(R), C.byref(S), C.byref(P)))
        return P.value

    def join_aggregate(self, keyR: Col, valR: Col | None, keyS: Col, valS: Col | None) -> tuple[int, int, int]:
        """(pairs, sum of valR x S partners, sum of valS x R partners) of two base columns"""
        out = (C.c_uint64 * 3)()
        self._chk(self.lib.qe_join_aggregate(self.h, keyR, valR if valR is not None else Col(None, 0), keyS,
                                             valS if valS is not None else Col(None, 0), out))
        return out[0], out[1], out[2]

    def checksum_weighted(self, col: Col, p: Pairs) -> int:
        s = C.c_uint64()
        self._chk(self.lib.qe_checksum_weighted(self.h, col, C.byref(p), C.byref(s)))
        return s.value

    def set_materialize_limit(self, pairs: int) -> None:
        self._chk(self.lib.qe_set_materialize_limit(self.h, pairs))

    def checksum(self, col: Col, rows: List | None) -> int:
        s = C.c_uint64()
        self._chk(self.lib.qe_checksum(self.h, col, C.byref(rows) if rows is not None else None, C.byref(s)))
        return s.value

    # ---- multi-GPU plan primitives ----
    def partition(self, keys_ptr: int, n: int, col_ptrs: list[int], nparts: int, out_keys_ptr: int,
                  out_col_ptrs: list[int]) -> list[int]:
        counts = (C.c_uint64 * nparts)()
        cols = (C.c_void_p * max(1, len(col_ptrs)))(*col_ptrs)
        ocols = (C.c_void_p * max(1, len(out_col_ptrs)))(*out_col_ptrs)
        self._chk(self.lib.qe_partition(self.h, keys_ptr, n, cols, len(col_ptrs), nparts, counts, out_keys_ptr,
                                        ocols))
        return list(counts)

    def filter_scan_range(self, col: Col, start: int, end: int, op: str, v: int) -> List:
        l = List()
        self._chk(self.lib.qe_filter_scan_range(self.h, col, start, end, op.encode(), v, C.byref(l)))
        return l

    def filter_scan2_range(self, col1: Col, op1: str, v1: int, col2: Col, op2: str, v2: int, start: int,
                           end: int) -> List:
        l = List()
        self._chk(self.lib.qe_filter_scan2_range(self.h, col1, op1.encode(), v1, col2, op2.encode(), v2, start, end,
                                                 C.byref(l)))
        return l

    def iota(self, start: int, n: int) -> List:
        l = List()
        self._chk(self.lib.qe_iota(self.h, start, n, C.byref(l)))
        return l

    def take_u32(self, src_ptr: int, idx: List) -> List:
        l = List()
        self._chk(self.lib.qe_take_u32(self.h, src_ptr, C.byref(idx), C.byref(l)))
        return l

    def join_indices(self, a_ptr: int, na: int, b_ptr: int, nb: int) -> tuple[List, List]:
        ia, ib = List(), List()
        self._chk(self.lib.qe_join_indices(self.h, a_ptr, na, b_ptr, nb, C.byref(ia), C.byref(ib)))
        return ia, ib

    def bucket_select(self, col: Col, nparts: int, part: int, heavy=None) -> Pairs:
        """(key, rowid) pairs of the base column's hash bucket `part` (heavy keys left out)"""
        h = np.ascontiguousarray(heavy if heavy is not None else np.zeros(0, np.uint64), dtype=np.uint64)
        p = Pairs()
        self._chk(self.lib.qe_bucket_select(self.h, col, nparts, part, h.ctypes.data if h.size else None, h.size,
                                            C.byref(p)))
        return p

    def partition_columns(self, nparts: int, part: int):
        """the partitioned layout for the plan at nparts ranks (qe_partition_columns): each base column
        a partitioned join reads as a whole side keeps this rank's hash bucket from its first use on"""
        self._chk(self.lib.qe_partition_columns(self.h, nparts, part))

    def heavy_stats(self, keys: Col, start: int, end: int, heavy, vals: Col | None = None, weights=None):
        """-> (counts per heavy key over rows [start, end), weighted value sum mod 2^64 or None)"""
        h = np.ascontiguousarray(heavy, dtype=np.uint64)
        counts = np.zeros(h.size, dtype=np.uint64)
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.uint64)
        s = C.c_uint64()
        self._chk(self.lib.qe_heavy_stats(self.h, keys, start, end, h.ctypes.data if h.size else None, h.size,
                                          vals if vals is not None else Col(), w.ctypes.data if w is not None else None,
                                          counts.ctypes.data if h.size else None, C.byref(s)))
        return counts, (s.value if w is not None else None)

    def sync(self):
        self._chk(self.lib.qe_sync(self.h))

    def mem_stats(self) -> tuple[int, int]:
        a, b = C.c_uint64(), C.c_uint64()
        self._chk(self.lib.qe_mem_stats(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def load_stats(self) -> tuple[float, float]:
        """(seconds, bytes) of every host -> HBM relation load so far (PCIe included)"""
        a, b = C.c_double(), C.c_double()
        self._chk(self.lib.qe_load_stats(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    # ---- profiling ----
    def set_profiling(self, on: bool):
        self._chk(self.lib.qe_set_profiling(self.h, 1 if on else 0))

    def set_profiling_only(self, stage: str | None):
        self._chk(self.lib.qe_set_profiling_only(self.h, stage.encode() if stage else None))

    def reset_stats(self):
        self._chk(self.lib.qe_reset_stats(self.h))

    def kernel_stats(self) -> dict:
        n = self._chk(self.lib.qe_kernel_stats(self.h, None, 0))
        arr = (KStat * max(1, n))()
        self._chk(self.lib.qe_kernel_stats(self.h, arr, n))
        return {arr[i].name.decode(): {"launches": arr[i].launches, "ms": arr[i].total_ms,
                                       "alg_bytes": arr[i].alg_bytes} for i in range(n)}


def comm_unique_id() -> bytes:
    """rank 0: the RCCL bootstrap id (128 bytes) every rank passes to Comm"""
    lib = load_library()
    b = C.create_string_buffer(128)
    rc = lib.qe_comm_unique_id(b)
    if rc != 0:
        raise QEError(rc, "ncclGetUniqueId failed")
    return b.raw


class Comm:
    """an RCCL communicator on a ctx's device (qe_comm_init): one rank per GPU"""

    def __init__(self, ctx: Ctx, nranks: int, rank: int, uid: bytes):
        self.ctx, self.lib = ctx, ctx.lib
        h = C.c_void_p()
        ctx._chk(self.lib.qe_comm_init(ctx.h, nranks, rank, uid, C.byref(h)))
        self.h = h
        self.nranks, self.rank = nranks, rank

    def allreduce(self, vals) -> list[int]:
        a = (C.c_uint64 * len(vals))(*[int(v) & ((1 << 64) - 1) for v in vals])
        self.ctx._chk(self.lib.qe_allreduce_u64(self.ctx.h, self.h, a, len(vals)))
        return list(a)

    def shuffle(self, keys_ptr: int, n: int, col_ptrs: list[int]):
        """qe_shuffle_pairs -> (keys ptr, [col ptrs], n) in ctx buffers (free with ctx.buffer_free)"""
        cols = (C.c_void_p * max(1, len(col_ptrs)))(*col_ptrs)
        ok, oc, on = C.c_void_p(), (C.c_void_p * max(1, len(col_ptrs)))(), C.c_uint64()
        self.ctx._chk(self.lib.qe_shuffle_pairs(self.ctx.h, self.h, keys_ptr, n, cols, len(col_ptrs), C.byref(ok),
                                                oc, C.byref(on)))
        return ok.value, [oc[i] for i in range(len(col_ptrs))], on.value

    def stats(self) -> tuple[int, int]:
        x, b = C.c_uint64(), C.c_uint64()
        self.lib.qe_comm_stats(self.h, C.byref(x), C.byref(b))
        return x.value, b.value

    def close(self):
        if self.h:
            self.lib.qe_comm_fini(self.h)
            self.h = None


class LocalComms:
    """qe_comm_init_local: in-process ranks over `ctxs` (e.g. Ctx.workers on one GPU); run() drives
    qe_run_queries_dist on every rank from its own host thread (ctypes releases the GIL)"""

    def __init__(self, ctxs: list[Ctx]):
        self.ctxs, self.lib = ctxs, ctxs[0].lib
        arr = (C.c_void_p * len(ctxs))(*[c.h for c in ctxs])
        out = (C.c_void_p * len(ctxs))()
        ctxs[0]._chk(self.lib.qe_comm_init_local(arr, len(ctxs), out))
        self.comms = []
        for i, c in enumerate(ctxs):
            cm = Comm.__new__(Comm)
            cm.ctx, cm.lib, cm.h, cm.nranks, cm.rank = c, self.lib, C.c_void_p(out[i]), len(ctxs), i
            self.comms.append(cm)

    def run(self, text: str) -> list:
        """per rank: (stdout, status, refused) or the QEError it raised"""
        import threading
        res = [None] * len(self.ctxs)

        def go(r):
            try:
                self.lib.qe_bind_thread(self.ctxs[r].h)
                res[r] = self.ctxs[r].run_dist(text, self.comms[r])
            except QEError as e:
                res[r] = e
        th = [threading.Thread(target=go, args=(r,)) for r in range(len(self.ctxs))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return res

    def bytes_sent(self) -> int:
        return sum(c.stats()[1] for c in self.comms)

    def close(self):
        for c in self.comms:
            c.close()

