"""Roofline record of the timed trace kernel from rocprofv3 runs of one bench command, and its
re-check from the committed record alone.

The trace kernel is a divergent, pointer-chasing path (no MFMA). Its roof is
stated against HBM as the contract asks (`bound: "hbm"`), with the MEASURED HBM bytes — not the
algorithmic §8(d) bytes, which small scenes serve from LDS — and beside it the resource that
actually binds, computed from PMC counters the same way for every workload:

  clock_hz        = GRBM_GUI_ACTIVE / 8 XCDs / duration      (GRBM_GUI_ACTIVE sums the XCDs)
  valu_issue_frac = SQ_INSTS_VALU / (CUs * 4 SIMDs * 0.5 wave-instr/clk * clock_hz * duration)
  lane_util       = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)
  fp32_lane_frac  = valu_issue_frac * lane_util               (fraction of the FP32 lane throughput)
  td_busy_frac    = TD_TD_BUSY_sum / CUs / (GRBM_GUI_ACTIVE / 8)   (mean busy fraction of a CU's TD)
  hbm_frac        = (2 * FETCH_SIZE + WRITE_SIZE) KiB * 1024 / duration / 8e12   (MI355X_MICROARCH.md)
  valu_lane_ops   = SQ_INSTS_VALU * 64 * lane_util           (useful FP32 lane-operations per launch)
  valu_peak_gops  = CUs * 4 SIMDs * 0.5 * 64 lanes * clock_hz / 1e9   (fp32_lane_frac = achieved / this)
  vmem_rd_gips    = SQ_INSTS_VMEM_RD / duration / 1e9        (vector-memory read wave-instructions/s)
  vmem_frac       = vmem_rd_gips / VMEM_PEAK_GIPS            (the measured dwordx4 gather ceiling,
                    profiles/r02_pair/td_width_bench.log mode 0: 2195 G lane-loads/s = 34.3 G/s)
  vmem_mix_frac   = vmem_rd_gips / VMEM_MIX_PEAK_GIPS[traversal]   (the ceiling for the traversal's
                    own node records, scripts/td_mix_bench.hip: 64-B wide records 40.6 G/s, 16-B
                    binary node rows 34.7 G/s; profiles/r04_tdmix/)
  vmem_mix_frac_resident = vmem_rd_gips / VMEM_MIX_PEAK_GIPS_RESIDENT[traversal]   (the same ceiling
                    measured at the kernels' own residency: 4 workgroups of 4 waves per CU, 24 of 64
                    lanes active; td_mix_bench 4 24, profiles/r05_tdmix/: 64-B records 41.85 G/s —
                    as at full occupancy, so that frac is not lost occupancy — 16-B rows 22.38)
  td_unstalled_frac = td_busy_frac * (1 - TD_TC_STALL_sum / TD_TD_BUSY_sum)   (cycles the TD moves
                    data rather than waits on the cache for it; agrees with vmem_mix_frac)

The roof that binds (bench.py `roofline.bound`): "valu" for LDS-mode kernels (the scene is in LDS;
issue of partly idle waves binds, frac = fp32_lane_frac), "vmem/TD" for HBM-mode kernels (node and
primitive records are L2-resident and return through TD, frac = vmem_mix_frac); hbm_frac beside it.
Every record carries `build`, the hash of the kernel sources and build flags it was measured on
(`source_hash`); bench.py uses a record's counts only for the build it describes.

usage:
  python scripts/roofline.py make --stats KT.csv --fetch DIR --write DIR [--pmc DIR] --workload W --out OUT.json
  python scripts/roofline.py check OUT.json [...]      # recompute every derived field, exit 1 on mismatch
  python scripts/roofline.py hash                       # source_hash() of this tree (the Makefile embeds it)
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import re
import sys

HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E (MI355X_MICROARCH.md)
# vector-memory read wave-instructions per second, measured: dependent random dwordx4 gathers over
# an L2-resident array (scripts/td_width_bench.hip, profiles/r02_pair/td_width_bench.log mode 0:
# 2195.0 G lane-loads/s / 64 lanes)
VMEM_PEAK_GIPS = 2195.0 / 64
# the same ceiling for the load each traversal order issues per node (scripts/td_mix_bench.hip,
# profiles/r04_tdmix/rates.log, L2-resident working set, TD busy 0.93-0.99; a 2 GiB working set is
# 1-25 % slower): the wide order's 64-B records are four dwordx4 of one record (40.60 G wave-instr/s),
# the binary orders' 16-B node rows one dwordx4 (34.71)
VMEM_MIX_PEAK_GIPS = {"wide": 40.60, "near": 34.71, "reference": 34.71}
# at the HBM-mode kernels' residency (4 workgroups per CU, 24 active lanes; L2-resident set)
VMEM_MIX_PEAK_GIPS_RESIDENT = {"wide": 41.85, "near": 22.38, "reference": 22.38}


def record_traversal(rec):
    m = re.search(r"traversal=(\w+)", rec.get("workload", ""))
    return m.group(1) if m and m.group(1) in VMEM_MIX_PEAK_GIPS else "near"
ROOT = __import__("pathlib").Path(__file__).resolve().parent.parent
_HIPCC_VERSION = None


def build_files(root=ROOT):
    """Every file the product library is built from: the Makefile, every source under csrc/ and
    the ABI header (the Makefile's HDR set and more)."""
    fs = ["julia-raytracer_amd/Makefile", "include/jtrace.h"]
    fs += sorted(str(p.relative_to(root)) for p in (root / "julia-raytracer_amd" / "csrc").iterdir() if p.is_file())
    return fs


def hipcc_version():
    global _HIPCC_VERSION
    if _HIPCC_VERSION is None:
        import subprocess
        try:
            out = subprocess.run(["/opt/rocm/bin/hipcc", "--version"], capture_output=True, text=True, timeout=60).stdout
            _HIPCC_VERSION = " ".join(l.strip() for l in out.splitlines() if "version" in l.lower())
        except (OSError, subprocess.SubprocessError):
            _HIPCC_VERSION = "unknown"
    return _HIPCC_VERSION


def source_hash(root=ROOT):
    """Hash of the library's sources, build flags and compiler version: identifies the build a
    record was measured on. The Makefile embeds the same hash in the library (jt_version)."""
    import hashlib
    h = hashlib.sha256()
    for f in build_files(root):
        h.update(f.encode())
        h.update((root / f).read_bytes())
    h.update(hipcc_version().encode())
    return h.hexdigest()[:16]


CUS = 256
XCDS = 8
KERNEL_RE = re.compile(r"(trace_kernel\w*<\d+, \d+, (?:true|false), 0, \d+, (?:true|false)>)")  # <.., WIDE>


def timed_kernel(stats_csv):
    best = None
    for r in csv.DictReader(open(stats_csv)):
        m = KERNEL_RE.search(r["Name"])
        if m and (best is None or float(r["TotalDurationNs"]) > best[0]):
            best = (float(r["TotalDurationNs"]), m.group(1), float(r["AverageNs"]), int(r["Calls"]))
    if best is None:
        raise SystemExit(f"no COUNT=0 trace kernel in {stats_csv}")
    return best[1], best[2], best[3]


def counter_means(d, kernel):
    """Per-dispatch sums of every counter of `kernel` (summed over the counter's dimensions),
    averaged over dispatches; plus the mean dispatch duration of those runs."""
    per = {}
    durs = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"].replace("(anonymous namespace)::", ""):
                continue
            key = (f, r["Dispatch_Id"])
            per.setdefault(r["Counter_Name"], {}).setdefault(key, 0.0)
            per[r["Counter_Name"]][key] += float(r["Counter_Value"])
            durs[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    means = {c: sum(v.values()) / len(v) for c, v in per.items()}
    return means, (sum(durs.values()) / len(durs) if durs else None)


def derive(rec):
    """Every derived field from the raw ones (used by make and by check)."""
    raw, out = rec["raw"], {}
    dur = rec["duration_ns"] * 1e-9
    traffic = 2.0 * raw["FETCH_SIZE"] * 1024.0 + raw["WRITE_SIZE"] * 1024.0
    out["traffic_bytes"] = traffic
    out["write_bytes"] = raw["WRITE_SIZE"] * 1024.0
    out["hbm_gbs"] = traffic / dur / 1e9
    out["hbm_frac"] = traffic / dur / HBM_PEAK
    pmc = rec.get("pmc") or {}
    if pmc.get("GRBM_GUI_ACTIVE") and pmc.get("pmc_duration_ns"):
        pd = pmc["pmc_duration_ns"] * 1e-9
        clk = pmc["GRBM_GUI_ACTIVE"] / XCDS / pd
        out["clock_ghz"] = clk / 1e9
        if pmc.get("SQ_INSTS_VALU"):
            out["valu_issue_frac"] = pmc["SQ_INSTS_VALU"] / (CUS * 4 * 0.5 * clk * pd)
        if pmc.get("SQ_THREAD_CYCLES_VALU") and pmc.get("SQ_ACTIVE_INST_VALU"):
            out["lane_util"] = pmc["SQ_THREAD_CYCLES_VALU"] / (64.0 * pmc["SQ_ACTIVE_INST_VALU"])
        if "valu_issue_frac" in out and "lane_util" in out:
            out["fp32_lane_frac"] = out["valu_issue_frac"] * out["lane_util"]
        if pmc.get("TD_TD_BUSY_sum"):  # summed over the 256 CUs' TD units
            out["td_busy_frac"] = pmc["TD_TD_BUSY_sum"] / CUS / (pmc["GRBM_GUI_ACTIVE"] / XCDS)
        if "lane_util" in out and pmc.get("SQ_INSTS_VALU"):
            out["valu_lane_ops"] = pmc["SQ_INSTS_VALU"] * 64.0 * out["lane_util"]
            out["valu_peak_gops"] = CUS * 4 * 0.5 * 64 * clk / 1e9
        gui = pmc["GRBM_GUI_ACTIVE"] / XCDS  # clock cycles of the launch
        if pmc.get("TA_TA_BUSY_sum"):
            out["ta_busy_frac"] = pmc["TA_TA_BUSY_sum"] / CUS / gui
        if pmc.get("TD_TC_STALL_sum") and pmc.get("TD_TD_BUSY_sum"):
            out["td_tc_stall_frac_of_busy"] = pmc["TD_TC_STALL_sum"] / pmc["TD_TD_BUSY_sum"]
        if pmc.get("TCC_HIT_sum") is not None and pmc.get("TCC_MISS_sum") is not None and \
                pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"] > 0:
            out["l2_hit_rate"] = pmc["TCC_HIT_sum"] / (pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"])
            out["l2_requests_per_launch"] = pmc["TCC_HIT_sum"] + pmc["TCC_MISS_sum"]
        if pmc.get("TCP_TOTAL_CACHE_ACCESSES_sum") and pmc.get("SQ_INSTS_VMEM_RD"):
            # L1 (TCP) cache accesses per vector-memory read wave-instruction (a divergent gather
            # touches one line per distinct address)
            out["l1_accesses_per_vmem_rd"] = pmc["TCP_TOTAL_CACHE_ACCESSES_sum"] / pmc["SQ_INSTS_VMEM_RD"]
        if pmc.get("TCP_TCC_READ_REQ_sum") is not None and pmc.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
            # L1 (TCP) locality: read requests the L1 sends on to L2 (its misses) per access and per
            # vector-memory read wave-instruction (the distinct lines a gather misses)
            out["l1_hit_rate"] = 1.0 - pmc["TCP_TCC_READ_REQ_sum"] / pmc["TCP_TOTAL_CACHE_ACCESSES_sum"]
            if pmc.get("SQ_INSTS_VMEM_RD"):
                out["l1_misses_per_vmem_rd"] = pmc["TCP_TCC_READ_REQ_sum"] / pmc["SQ_INSTS_VMEM_RD"]
        if pmc.get("TCP_PENDING_STALL_CYCLES_sum"):
            out["tcp_pending_stall_frac"] = pmc["TCP_PENDING_STALL_CYCLES_sum"] / CUS / gui
        if pmc.get("SQ_WAVE_CYCLES"):
            # where a resident wave's cycles go (disjoint, MI355X_MICROARCH.md rocprofv3 PMC slots):
            # issuing, parked on s_waitcnt / barrier (memory latency), or ready but not issued
            for k, name in (("SQ_ACTIVE_INST_ANY", "wave_active_frac"), ("SQ_WAIT_ANY", "wave_wait_frac"),
                            ("SQ_WAIT_INST_ANY", "wave_issue_stall_frac"), ("SQ_WAIT_INST_LDS", "wave_lds_stall_frac"),
                            ("SQ_ACTIVE_INST_SCA", "wave_salu_frac"), ("SQ_ACTIVE_INST_LDS", "wave_lds_frac")):
                if pmc.get(k) is not None:
                    out[name] = pmc[k] / pmc["SQ_WAVE_CYCLES"]
        if pmc.get("SQ_INSTS_VMEM_RD"):
            out["vmem_rd_per_launch"] = pmc["SQ_INSTS_VMEM_RD"]
            out["vmem_rd_gips"] = pmc["SQ_INSTS_VMEM_RD"] / pd / 1e9
            out["vmem_frac"] = out["vmem_rd_gips"] / VMEM_PEAK_GIPS
            out["vmem_mix_frac"] = out["vmem_rd_gips"] / VMEM_MIX_PEAK_GIPS[record_traversal(rec)]
            out["vmem_mix_frac_resident"] = out["vmem_rd_gips"] / VMEM_MIX_PEAK_GIPS_RESIDENT[record_traversal(rec)]
        if "td_busy_frac" in out and "td_tc_stall_frac_of_busy" in out:
            out["td_unstalled_frac"] = out["td_busy_frac"] * (1.0 - out["td_tc_stall_frac_of_busy"])
    return {k: round(v, 6) for k, v in out.items()}


def make(a):
    kernel, avg_ns, calls = timed_kernel(a.stats)
    f, _ = counter_means(a.fetch, kernel)
    w, _ = counter_means(a.write, kernel)
    if "FETCH_SIZE" not in f or "WRITE_SIZE" not in w:
        raise SystemExit("FETCH_SIZE / WRITE_SIZE of the timed kernel not found")
    rec = {"workload": a.workload, "kernel": kernel, "build": source_hash(), "duration_ns": avg_ns, "calls": calls,
           "raw": {"FETCH_SIZE": f["FETCH_SIZE"], "WRITE_SIZE": w["WRITE_SIZE"]}}
    if a.pmc:
        pmc, pdur = {}, []
        for d in sorted(glob.glob(f"{a.pmc}/p*/")):
            m, dd = counter_means(d, kernel)
            pmc.update(m)
            if dd:
                pdur.append(dd)
        if pdur:
            pmc["pmc_duration_ns"] = sum(pdur) / len(pdur)
        rec["pmc"] = pmc
    rec["derived"] = derive(rec)
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec["derived"]))


def check(paths):
    bad = 0
    for p in paths:
        rec = json.load(open(p))
        again = derive(rec)
        for k, v in again.items():
            if k not in rec["derived"]:  # a field added after this record was written
                continue
            if abs(rec["derived"][k] - v) > 1e-6 * max(1.0, abs(v)):
                print(f"{p}: {k} recorded {rec['derived'].get(k)} recomputed {v}")
                bad += 1
        if again["hbm_frac"] > 1.0:
            print(f"{p}: hbm_frac {again['hbm_frac']} > 1")
            bad += 1
        print(p, json.dumps(again))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    m = sub.add_parser("make")
    m.add_argument("--stats", required=True)
    m.add_argument("--fetch", required=True)
    m.add_argument("--write", required=True)
    m.add_argument("--pmc")
    m.add_argument("--workload", required=True)
    m.add_argument("--out", required=True)
    c = sub.add_parser("check")
    c.add_argument("paths", nargs="+")
    sub.add_parser("hash")
    a = ap.parse_args()
    if a.cmd == "hash":
        print(source_hash())
    else:
        make(a) if a.cmd == "make" else check(a.paths)
