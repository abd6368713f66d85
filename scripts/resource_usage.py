"""Resource usage of every production kernel instance (COUNT=0) of libjtrace_hip: VGPRs, spilled
VGPRs, scratch bytes per lane, occupancy, per launch configuration (csrc/jt_kernels.h
LaunchConfig), and the scratch stores inside the kernel's loops (spill write-back executed per
path or per query, not once per launch: the WRITE traffic the roofline records show). Compiles
csrc/jt_kv.hip once per configuration with -Rpass-analysis and once to ISA.
usage: python scripts/resource_usage.py [extra hipcc flags...]"""
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent / "julia-raytracer_amd"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-DJT_EXACT_MATH=1", "-fno-slp-vectorize", "-mllvm", "-sink-insts-to-avoid-spills=1", "-DJT_WAVES=4"]
NAMES = ["FT_NONE+LINL", "FT_ALL", "FT_MESH+LINL", "FT_MESH_ENV+NOIL", "FT_MESH_ENV_QUAD+LINL", "FT_ALL ovf", "FT_ALL ring32",
         "FT_NONE lsteps"]
NAMES += [n + " wide" for n in NAMES]  # configurations 8-15: the wide traversal


def usage(v, extra):
    out = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, f"-DJT_VARIANT={v}", "-c", "-o", "/dev/null",
                          "csrc/jt_kv.hip", "-Rpass-analysis=kernel-resource-usage"], cwd=PKG, capture_output=True,
                         text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark: ([\w \[\]/]+): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    asm = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, f"-DJT_VARIANT={v}", "--cuda-device-only", "-S",
                          "-o", "-", "csrc/jt_kv.hip"], cwd=PKG, capture_output=True, text=True).stdout
    for r in rows:
        r["loop_stores"] = loop_scratch_stores(asm, r["name"])
    return v, rows


def loop_scratch_stores(asm, name):
    """scratch_store instructions of one kernel that sit in a loop block ("in Loop:" / "Loop
    Header" comments of the basic block they belong to)."""
    i = asm.find(name + ":")
    if i < 0:
        return -1
    j = asm.find(".Lfunc_end", i)
    in_loop, n = False, 0
    for line in asm[i:j].splitlines():
        if re.match(r"^(\.LBB|; %bb)", line):
            in_loop = "Loop" in line
        elif line.lstrip().startswith("; =>") or "Parent Loop" in line:
            in_loop = True
        if in_loop and "scratch_store" in line:
            n += 1
    return n


def main():
    extra = sys.argv[1:]
    with ThreadPoolExecutor(7) as ex:
        res = list(ex.map(lambda v: usage(v, extra), range(len(NAMES))))
    print(f"{'config':22} {'kernel':16} {'sampler':7} {'VGPRs':>5} {'spill':>5} {'scratch':>7} {'occ':>3} {'loop stores':>11}")
    for v, rows in res:
        for r in rows:
            m = re.search(r"(trace_kernel\w*)ILi(\d)ELi(\d+)ELb(\d)ELi(\d)ELi(\d+)ELb(\d)E", r["name"])
            if not m or m.group(5) != "0":
                continue
            print(f"{NAMES[v]:22} {m.group(1):16} {m.group(2):7} {r.get('VGPRs', 0):5} {r.get('VGPRs Spill', 0):5} "
                  f"{r.get('ScratchSize [bytes/lane]', 0):7} {r.get('Occupancy [waves/SIMD]', 0):3} {r['loop_stores']:11}")


if __name__ == "__main__":
    main()
