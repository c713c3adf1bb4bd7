#!/bin/bash
# MFMA gap profile of the main loop of a kernel: compile one source with extra flags, print the
# VGPR count and, per MFMA of the largest loop, the VALU / transcendental / LDS instructions
# issued since the previous MFMA.  usage: scripts/isa_gaps.sh src.hip 'kernel-symbol-regex' [flags...]
set -e
src=$1; pat=$2; shift 2
d=$(mktemp -d)
cd "$d"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I"$GRAFT_ROOT/include" -I"$GRAFT_ROOT/numpyro_amd/csrc" "$@" \
  -x hip -c "$GRAFT_ROOT/numpyro_amd/csrc/$src" --save-temps -o x.o 2>/dev/null
S=$(ls *gfx950*.s)
start=$(grep -n "^${pat}:" "$S" | head -1 | cut -d: -f1)
end=$(awk -v s="$start" 'NR>s && /^.Lfunc_end/{print NR; exit}' "$S")
sed -n "${start},${end}p" "$S" > k.s
grep -m1 -A0 "\.vgpr_count\|NumVgprs" k.s || true
awk '/; NumVgprs|; Occupancy|; ScratchSize/' "$S" | head -0
# largest loop: between "Loop Header" label and its backward branch
python3 - k.s <<'PY'
import re, sys
lines = open(sys.argv[1]).read().splitlines()
labels = {l.split(':')[0]: i for i, l in enumerate(lines) if re.match(r'^\.LBB\d+_\d+:', l)}
best = None
for i, l in enumerate(lines):
    m = re.match(r'\s+s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        a = labels[m.group(2)]
        body = lines[a:i]
        n = sum(1 for x in body if 'mfma' in x)
        if best is None or n > best[0]:
            best = (n, a, i)
n, a, b = best
v = t = d = w = 0
gaps = []
for x in lines[a:b]:
    op = x.split()[0] if x.split() else ''
    if 'mfma' in op:
        gaps.append((v, t, d, w)); v = t = d = w = 0
    elif re.match(r'v_(exp|rcp|log|sqrt|rsq)', op): t += 1
    elif op.startswith('v_'): v += 1
    elif op.startswith('ds_'): d += 1
    elif 'waitcnt' in op: w += 1
print(f"loop lines {a}-{b}: {n} MFMA; VALU+trans per gap: " + " ".join(f"{g[0]}+{g[1]}" for g in gaps) + f" | tail {v}+{t}")
tot_v = sum(g[0] for g in gaps) + v; tot_t = sum(g[1] for g in gaps) + t
print(f"total VALU {tot_v}, transcendental {tot_t}")
PY
grep "\.vgpr_count" "$S" | head -0
awk -v p="$pat" '$0 ~ "\\.name:.*" && $0 ~ p {f=1} f && /\.vgpr_count/ {print "vgpr_count", $2; exit}' "$S"
rm -rf "$d"
