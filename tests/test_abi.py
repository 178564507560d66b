"""CPU-side checks of the C ABI boundary: libqe builds, loads, and exports every symbol
include/qe.h declares (no compute calls -- there is no GPU here)."""
import ctypes
import os
import subprocess

import pytest

from qe import lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "query-compiler-executor_amd")], check=True)
    return lib.load_library()


def test_header_declares_the_hot_path():
    syms = lib.declared_symbols()
    for s in ["qe_filter_scan", "qe_filter_refine", "qe_gather_pairs", "qe_sort_pairs", "qe_merge_join",
              "qe_scan_join", "qe_driver_counts", "qe_join_payloads", "qe_checksum", "qe_run_queries"]:
        assert s in syms


def test_library_exports_every_declared_symbol(built):
    missing = [s for s in lib.declared_symbols() if not hasattr(built, s)]
    assert not missing, missing


def test_abi_version(built):
    assert built.qe_abi_version() == 1


def test_queries_binary_built(built):
    assert os.access(os.path.join(ROOT, "query-compiler-executor_amd", "build", "queries"), os.X_OK)


def test_library_is_gfx950_code(built):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib.LIB_PATH],
                         capture_output=True, text=True, cwd="/tmp")
    assert "gfx950" in out.stdout + out.stderr


def test_no_gpu_means_loud_failure(built):
    # this container has no GPU: the native path must refuse, not fall back
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(lib.QEError):
        lib.Ctx(0)


def test_plan_header_exports(built):
    """include/qe_plan.h: the partitioned plan is in libqe and, alone, in libqeplan.so (the CPU
    tests' build of the same C)"""
    hdr = os.path.join(ROOT, "include", "qe_plan.h")
    syms = lib.declared_symbols(hdr)
    assert {"qe_plan_run_text", "qe_plan_check_text", "qe_plan_why"} <= set(syms)
    plan = ctypes.CDLL(os.path.join(ROOT, "query-compiler-executor_amd", "build", "libqeplan.so"))
    for s in syms:
        assert hasattr(built, s) and hasattr(plan, s), s


def test_multi_gpu_abi_declared():
    """the multi-GPU half of the boundary"""
    syms = set(lib.declared_symbols())
    assert {"qe_comm_init", "qe_shuffle_pairs", "qe_allreduce_u64", "qe_run_queries_dist"} <= syms
