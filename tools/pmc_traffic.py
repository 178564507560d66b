#!/usr/bin/env python3
"""HBM bytes per launch per bench stage from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py --fetch DIR --write DIR --out profiles/r01_traffic.json \
        --command "<the rocprofv3 commands>"

Counters (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in KiB and count the
L2's memory-side requests; on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide coalesced
streaming read, so it is doubled here (`fetch_corrected`); WRITE_SIZE is taken as is.  The two
counters cannot share a pass, hence two runs of the same command.

Kernels are mapped to the stage names libqe's own timers use (bench.py "stages").  One libqe
stage timer (`Timed`) may cover several dispatches (bucket_join_sums = the sums kernel + its
reduce; sort_hist = the histogram + its column sums), so per-dispatch averages are NOT comparable
with the bench's per-`Timed` launches: the comparable figure is bytes PER QUERY
(`hbm_bytes_per_query` = all of the stage's dispatches in the profiled run / the queries it ran,
`--queries`; bench.py's c3 loop with `--steps S --warmup W` runs W + 2 S of them).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

# demangled kernel name -> bench stage (first match wins)
STAGES = [
    (r"radix_pass_kernel<unsigned long, \d, \d, true, \d+, \d+, \d+, true, [123]\b", "sort_pass_carry"),
    (r"tl_pass2_kernel<unsigned long, [12]\b", "sort_pass_carry"),
    # a 64-bit key sort's first pass reading the base column's u32 copy (unstable: deferred sorts only)
    (r"radix_pass_kernel<unsigned int, \d, \d, true, \d+, \d+, \d+, true, [123], true(, \d+)?>", "sort_pass_carry"),
    (r"radix_pass_kernel<unsigned int, \d, \d, true, \d+, \d+, \d+, true, 0, true(, \d+)?>", "sort_pass_k64v32"),
    (r"radix_pass_kernel<unsigned long, \d, \d, true", "sort_pass_k64v32"),
    (r"radix_pass_kernel<unsigned int, \d, \d, true", "sort_pass_k32v32"),
    (r"radix_pass_kernel<unsigned long, \d, \d, false", "sort_pass_k64"),
    (r"radix_pass_kv_kernel<unsigned long", "sort_pass_k64v32"),
    (r"radix_pass_kv_kernel<unsigned int", "sort_pass_k32v32"),
    (r"tl_pass2_kernel<unsigned long(, 0\b[^>]*)?>", "sort_pass_k64v32"),
    (r"tl_pass2_kernel<unsigned int(, 0\b[^>]*)?>", "sort_pass_k32v32"),
    (r"digit_hist_kernel|digit_scan_kernel|tl_hist_kernel|tl_hist8_kernel|tl_hist_tiles_kernel|tl_gfold_kernel|tl_bstart_kernel|tl_scan_kernel|tl_scan8_kernel", "sort_hist"),
    (r"cs_reduce_kernel|cs_top_kernel|cs_apply_kernel|cs_single_kernel", "sort_scan"),
    (r"tl_local_kernel", "sort_local"),
    (r"bucket_select_kernel", "bucket_select"),
    (r"part_count_kernel", "partition_count"),
    (r"part_scatter_kernel", "partition"),
    (r"take_u32_kernel", "take_u32"),
    (r"heavy_stats_kernel", "heavy_stats"),
    (r"key_bits_kernel", "sort_keybits"),
    (r"tl_hjoin_sums_kernel|tl_hjoin_sums_small_kernel|hjoin_sums_reduce_kernel", "bucket_join_sums"),
    (r"gather_u32_kernel", "gather_values"),
    (r"sum_u32_kernel", "checksum"),
    (r"tl_hjoin_kernel|tl_hjoin_chain_kernel", "bucket_join"),
    (r"mj_fused", "mj_fused"),
    (r"mj_partition", "mj_partition"),
    (r"mj_tile<1>", "mj_write"),
    (r"tl_gather_hist_kernel<true>|widen_u32_kernel", "widen_keys"),
    (r"gather_keys_kernel|tl_gather_hist_kernel", "gather_keys"),
    (r"expand_kernel<1>", "payload_expand"),
    (r"expand_kernel<0>|tile_scan_kernel", "payload_count"),
    (r"NonzeroPairsOp", "payload_prune"),
    (r"nonzero_bitmap_kernel", "payload_bitmap"),
    (r"FilterScanOp|FilterScan2Op|wscan_kernel|uscan_kernel", "filter_scan"),
    (r"zip_take_kernel", "take_u32"),
    (r"ag_tile_kernel|ag_reduce_kernel|ab_bucket_kernel|ab_sum3_kernel", "agg_count"),
    (r"ab_big_count_kernel|ab_big_look_kernel", "agg_big"),
    (r"ag_split_kernel", "agg_split"),
    (r"FilterRefineOp", "filter_refine"),
    (r"ScanJoinOp", "scan_join"),
    (r"scatter_match_kernel", "driver_scatter"),
    (r"checksum_kernel", "checksum"),
    (r"gen_column_kernel", "gen_column"),
]


# C5 (the aggregate join): every radix pass is one of its word sorts / partition passes
STAGES_C5 = [(r"radix_pass_kernel|tl_pass2_kernel", "sort_pass_agg")]


def stage_of(kname: str, workload: str = "c3"):
    for pat, st in (STAGES_C5 if workload == "c5" else []) + STAGES:
        if re.search(pat, kname):
            return st
    return None


def read_counter(d: str, counter: str):
    """{dispatch_id: (kernel_name, value)} from a rocprofv3 counter_collection csv under d."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    out = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                did = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                name = row.get("Kernel_Name", "")
                v = float(row["Counter_Value"])
                prev = out.get(did)
                out[did] = (name, v + (prev[1] if prev else 0.0))   # summed over dimensions
    return out


def per_stage(disp, workload="c3"):
    acc = defaultdict(lambda: [0.0, 0, set()])
    for name, v in disp.values():
        st = stage_of(name, workload)
        if st is None:
            continue
        a = acc[st]
        a[0] += v
        a[1] += 1
        a[2].add(re.sub(r"\(.*", "", name)[:120])
    return acc


def infer_queries(command: str):
    """bench.py's c3 plan loop runs warmup + 2 x steps queries (the stage table + the timed loop)"""
    m_s = re.search(r"--steps (\d+)", command or "")
    m_w = re.search(r"--warmup (\d+)", command or "")
    if not m_s or "bench.py" not in command or "--workload c4" in command or "--workload c5" in command:
        return None
    return (int(m_w.group(1)) if m_w else 2) + 2 * int(m_s.group(1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--command", default="")
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--queries", type=int, default=None,
                    help="queries the profiled command ran (bench.py c3 plan: warmup + 2 x steps)")
    a = ap.parse_args()
    q = a.queries or infer_queries(a.command)
    f = per_stage(read_counter(a.fetch, "FETCH_SIZE"), a.workload)
    w = per_stage(read_counter(a.write, "WRITE_SIZE"), a.workload)
    kern = {}
    for st in sorted(set(f) | set(w)):
        fk, fn, names = f.get(st, [0.0, 0, set()])
        wk, wn, names2 = w.get(st, [0.0, 0, set()])
        fpl = fk * 1024.0 / fn if fn else None
        wpl = wk * 1024.0 / wn if wn else None
        hbm = (2.0 * fpl if fpl is not None else 0.0) + (wpl or 0.0)
        kern[st] = {"hbm_bytes_per_launch": round(hbm), "fetch_raw_bytes_per_launch": round(fpl) if fpl else None,
                    "fetch_corrected_bytes_per_launch": round(2 * fpl) if fpl else None,
                    "write_bytes_per_launch": round(wpl) if wpl else None, "launches_fetch_pass": fn,
                    "launches_write_pass": wn, "kernels": sorted(names | names2),
                    "hbm_bytes_per_query": round((2.0 * fk + wk) * 1024.0 / q) if q else None,
                    "dispatches_per_query": round(fn / q, 3) if q else None}
    doc = {"command": a.command, "workload": a.workload, "queries": q,
           "units": "bytes per launch; FETCH_SIZE/WRITE_SIZE KiB x 1024",
           "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md HBM section); WRITE_SIZE as is",
           "kernels": kern}
    with open(a.out, "w") as fo:
        json.dump(doc, fo, indent=1)
    for st, k in sorted(kern.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
        print(f"{st:20s} {k['hbm_bytes_per_launch'] / 1e9:8.3f} GB/launch  (fetch x2 {k['fetch_corrected_bytes_per_launch']}, "
              f"write {k['write_bytes_per_launch']}, n={k['launches_fetch_pass']})")


if __name__ == "__main__":
    main()
