#!/bin/bash
# SURVEY.md section 5 sanitizer row, CPU side: AddressSanitizer + UndefinedBehaviorSanitizer builds of
# the host code of libcsa_legacy.so (csa_legacy.hip's host half -- instance upload, ABI argument checks,
# plans, the csa_legacy_sample pipeline bookkeeping -- and legacy_mt.cpp, the MT19937 draw) and of the C
# oracle, then the CPU test suite (pytest -m "not gpu": ABI symbol loads, the MT product path and the
# oracle against every golden) under them.  Device code is not instrumented (no GPU sanitizer on this
# pool): -fsanitize goes to the host compilation only (-Xarch_host).  Both builds use clang's runtime,
# preloaded into the uninstrumented python; the oracle is built without OpenMP (one ASan runtime, no
# second OpenMP runtime beside torch's).  Usage (repo root, CPU container): bash tools/asan_host.sh [log]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/exp/asan; mkdir -p "$OUT"
LOG=${1:-$ROOT/profiles/r05_asan_host_tests.log}
CLANG_RT=$(ls -d /opt/rocm/llvm/lib/clang/*/lib/linux | head -1)
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer
     -Xarch_host -fno-sanitize-recover=undefined)
hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -Wall "${SAN[@]}" -shared-libsan \
    -o "$OUT/libcsa_legacy.so" "$ROOT/citizensassemblies-replication_amd/csrc/csa_legacy.hip" \
    "$ROOT/citizensassemblies-replication_amd/csrc/legacy_mt.cpp"
/opt/rocm/llvm/bin/clang -O1 -g -fPIC -shared -std=c11 -Wall -fsanitize=address,undefined -fno-omit-frame-pointer \
    -fno-sanitize-recover=undefined -shared-libsan -Wno-unknown-pragmas -o "$OUT/liblegacy_oracle.so" \
    "$ROOT/oracle/legacy_oracle.c"
cd "$ROOT"
{
  echo "# $(date -u +%FT%TZ) ASan+UBSan host builds: $OUT/libcsa_legacy.so, $OUT/liblegacy_oracle.so"
  echo "# runtime: $CLANG_RT/libclang_rt.asan-x86_64.so (LD_PRELOAD), ASAN_OPTIONS=detect_leaks=0"
  LD_PRELOAD=$CLANG_RT/libclang_rt.asan-x86_64.so ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 CSA_LIB=$OUT/libcsa_legacy.so CSA_ORACLE_LIB=$OUT/liblegacy_oracle.so \
      python -m pytest tests -m "not gpu" -q -p no:cacheprovider 2>&1
  # which builds that python actually mapped (the instrumented ones, and the ASan runtime)
  LD_PRELOAD=$CLANG_RT/libclang_rt.asan-x86_64.so ASAN_OPTIONS=detect_leaks=0 CSA_LIB=$OUT/libcsa_legacy.so \
  CSA_ORACLE_LIB=$OUT/liblegacy_oracle.so python -c "
import importlib, sys
sys.path.insert(0, '.')
importlib.import_module('citizensassemblies-replication_amd._native').lib()
from oracle import coracle; coracle.lib()
maps = {l.split()[-1] for l in open('/proc/self/maps') if l.split()[-1].endswith('.so')}
print('# mapped:', sorted(m for m in maps if 'asan' in m or 'csa_legacy' in m or 'legacy_oracle' in m))"
} > "$LOG"
tail -3 "$LOG"
