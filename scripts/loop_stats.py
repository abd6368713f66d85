"""Instruction mix of the traversal loop (the Depth=2 loop holding the s_bcnt1 ballots) of one
kernel in a hipcc -S listing. usage: python scripts/loop_stats.py <file.s> [kernel-prefix]"""
import collections
import re
import sys

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "_ZN12_GLOBAL__N_116trace_kernel_ldsILi1ELi16ELi0E"
s = open(path).read().split("\n")
start = next(i for i, l in enumerate(s) if l.startswith(name))
end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
k = s[start:end]
# the traversal loop: the innermost loop around the first run of >= 3 s_bcnt1 (the step ballots)
bc = [i for i, l in enumerate(k) if "s_bcnt1" in l]
b = next(bc[n] for n in range(len(bc) - 2) if bc[n + 2] - bc[n] < 40)
h = next(i for i in range(b, 0, -1) if "This Loop Header:" in k[i])
hdr = next(re.match(r"\.LBB\d+_\d+", k[i]).group(0) for i in range(h, 0, -1) if k[i].startswith(".LBB"))
body = [l for l in k[h - 1:] ]
# the loop ends at the last line that is "in Loop: Header=<hdr>" region: take blocks whose
# comment names this header (or deeper loops nested in it)
blocks, cur, keep = [], [], False
for l in k:
    m = re.match(r"(\.LBB\d+_\d+|; %bb\.\d+):", l)
    if m:
        blocks.append((keep, cur))
        cur = []
        tag = hdr[4:]
        keep = (f"Header=BB{tag} " in l or l.startswith(hdr + ":") or f"Parent Loop BB{tag} " in l)
    cur.append(l)
blocks.append((keep, cur))
ins = [l.strip() for kp, c in blocks if kp for l in c if re.match(r"\s+[a-z_0-9]+", l) and not l.strip().startswith(";")]
cnt = collections.Counter(l.split()[0] for l in ins)
tot = collections.Counter()
for op, n in cnt.items():
    tot["valu" if op.startswith("v_") else "salu" if op.startswith("s_") else op.split("_")[0]] += n
print(hdr, dict(tot), "total", sum(cnt.values()))
for op, n in cnt.most_common(25):
    print(f"  {n:4d} {op}")

if len(sys.argv) > 3:  # per-block breakdown
    for kp, c in blocks:
        if not kp:
            continue
        ops = [l.strip().split()[0] for l in c if re.match(r"\s+[a-z_0-9]+", l) and not l.strip().startswith(";")]
        nm = sum(1 for o in ops if o.startswith("v_mov"))
        print(f"{c[0][:40]:42s} valu {sum(1 for o in ops if o.startswith('v_')):4d} mov {nm:3d} salu {sum(1 for o in ops if o.startswith('s_')):3d} ds {sum(1 for o in ops if o.startswith('ds_')):2d}")
