#!/bin/bash
# Host sanitizer build (CPU only; never run on the GPU box): AddressSanitizer + UBSan on the
# threaded host code — the MAF reader (csrc/maf.cpp), the result writers (csrc/writers.cpp),
# the plan builder and host-block packing (csrc/planner.cpp, host_io.cpp, capi.cpp), the V_lst
# scan extension (csrc/blocks_ext.c) and the CPU restatement (oracle/hmm_oracle.c) — then the
# CPU tests that drive them: tests/test_maf.py, test_writers.py, test_capi.py (the V_lst scan
# and symbol packing), test_partition.py (the planner) and test_oracle.py.
#   bash scripts/asan_host.sh [log]      (default log: profiles/r6_asan_host.log)
# The device code of the library is built as usual (sanitizer flags on the host side only);
# the sanitized objects go to $OUT (default /tmp/itr_asan), never into the package.
set -euo pipefail
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=${OUT:-/tmp/itr_asan}
LOG=$(realpath -m "${1:-profiles/r6_asan_host.log}")
mkdir -p "$OUT"
HIPCC=/opt/rocm/bin/hipcc
CLANG=/opt/rocm/lib/llvm/bin/clang
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
HSAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"
CSAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"
COMMON="--offload-arch=gfx950 -O1 -std=c++17 -fPIC -fvisibility=hidden"
CSRC=itrails_amd/csrc
pids=()
objs=()
for f in maf.cpp writers.cpp planner.cpp host_io.cpp capi.cpp; do  # host translation units
  o=$OUT/${f%.*}.o; objs+=("$o")
  $HIPCC $COMMON $HSAN -c $CSRC/$f -o "$o" & pids+=($!)
done
for f in hmm_sweeps.hip mfma_sweeps.hip wave_sweeps.hip dense.hip vanloan.hip emission.hip rows.hip prune_vit.hip; do
  o=$OUT/${f%.*}.o; objs+=("$o")
  case $f in hmm_sweeps.hip|mfma_sweeps.hip|wave_sweeps.hip|prune_vit.hip) X=-fno-honor-nans;; *) X=;; esac
  $HIPCC $COMMON -O3 $X -c $CSRC/$f -o "$o" 2>/dev/null & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$OUT/libitrails_hip_asan.so"
PYINC=$(python3 -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
NPINC=$(python3 -c 'import numpy; print(numpy.get_include())')
EXT=$(python3 -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
$CLANG -O1 $CSAN -shared -fPIC -I"$PYINC" -I"$NPINC" $CSRC/blocks_ext.c -o "$OUT/_blocks$EXT"
$CLANG -O1 $CSAN -fopenmp -shared -fPIC -std=c11 oracle/hmm_oracle.c -o "$OUT/liboracle_asan.so" -lm
{
  echo "# scripts/asan_host.sh  $(date -u +%FT%TZ)  $(git rev-parse --short HEAD 2>/dev/null)"
  echo "# runtime: $RT"
  echo "# host flags: $HSAN / $CSAN"
  for f in "$OUT/libitrails_hip_asan.so" "$OUT/_blocks$EXT" "$OUT/liboracle_asan.so"; do
    echo "# $(basename "$f"): $(nm -D "$f" | grep -c '__asan_report') ASan report hooks," \
         "$(nm -D "$f" | grep -c '__ubsan_handle') UBSan handlers referenced"
  done
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:strict_string_checks=1:detect_stack_use_after_return=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  LD_PRELOAD="$RT" ITR_LIB="$OUT/libitrails_hip_asan.so" ITR_BLOCKS_EXT="$OUT/_blocks$EXT" \
  ITR_ORACLE_LIB="$OUT/liboracle_asan.so" OMP_NUM_THREADS=8 \
    python3 -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_maf.py tests/test_writers.py \
      tests/test_capi.py tests/test_partition.py tests/test_oracle.py 2>&1
  echo "# exit status ${PIPESTATUS[0]}"
} | tee "$LOG"
grep -q "passed" "$LOG" && ! grep -qE "ERROR: AddressSanitizer|runtime error:|failed" "$LOG"
