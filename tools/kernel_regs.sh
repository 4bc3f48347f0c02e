#!/bin/bash
# Register / LDS / spill report of the gfx950 code object in a built library (default: the in-tree
# libcsa_legacy.so).  Usage: bash tools/kernel_regs.sh [regex of kernel names] [library]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LIB=${2:-$ROOT/citizensassemblies-replication_amd/libcsa_legacy.so}
PAT=${1:-.}
TMP=$(mktemp -d); trap 'rm -rf "$TMP"' EXIT
cp "$LIB" "$TMP/lib.so"
(cd "$TMP" && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading lib.so > /dev/null)
CO=$(ls "$TMP"/lib.so.*gfx950*)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$CO" | python3 -c "
import re, sys
txt = sys.stdin.read()
for blk in re.split(r'\n  - \.', txt)[1:]:
    f = dict(re.findall(r'\.?([a-z_]+):\s+(\S+)', blk))
    name = f.get('name', '')
    if not re.search(sys.argv[1], name): continue
    print('%-90s vgpr %4s agpr %4s spill %3s lds %6s scratch %4s' % (name[:90], f.get('vgpr_count'), f.get('agpr_count'),
          f.get('vgpr_spill_count'), f.get('group_segment_fixed_size'), f.get('private_segment_fixed_size')))
" "$PAT"
