#!/bin/bash
# Static analysis of the native sources (`make lint`): the clang static
# analyzer (core, cplusplus, deadcode, unix, security checkers) over every
# host C++ file and over the host side of every HIP file, plus a strict-warning
# syntax pass (-Wshadow -Wcast-qual -Wnon-virtual-dtor ...).  Role of the
# reference's cpplint -> cppcheck-XML script (/root/reference/fullcheck_xml.sh:3).
# Findings go to build/lint/report.txt; exit status 1 when there are any.
# Copyright 2026 veles.simd_amd authors. Apache-2.0.
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CLANG=${CLANG:-/opt/rocm/lib/llvm/bin/clang++}
OUT=$ROOT/build/lint
mkdir -p "$OUT"
REPORT=$OUT/report.txt
: > "$REPORT"
INC=(-std=c++17 -I"$ROOT" -I"$ROOT/include" -DVELES_SIMD_IMPLEMENTATION)
STRICT=(-Wall -Wextra -Wshadow -Wcast-qual -Wnon-virtual-dtor -Wmissing-declarations
        -Wno-unused-parameter -Wno-unused-command-line-argument)

cd "$ROOT"
CPP=$(ls csrc/*/*.cpp)
HIP=$(ls csrc/kernels/*.hip)
jobs=${LINT_JOBS:-8}

analyze() {  # file [extra flags...]
  local f=$1; shift
  "$CLANG" --analyze "${INC[@]}" "$@" -Xanalyzer -analyzer-output=text \
      -o /dev/null "$f" 2>&1 | grep -E "warning:|error:" || true
}
strict() {
  local f=$1; shift
  "$CLANG" -fsyntax-only "${INC[@]}" "${STRICT[@]}" "$@" "$f" 2>&1 |
      grep -E "warning:|error:" || true
}
export -f analyze strict
export CLANG ROOT
export INC_S="${INC[*]}" STRICT_S="${STRICT[*]}"

{
  # every file as hipcc compiles it (host pass only)
  for f in $CPP $HIP; do echo "$f"; done | xargs -P "$jobs" -I{} bash -c \
    'INC=($INC_S); STRICT=($STRICT_S); analyze {} -x hip --offload-arch=gfx950 --cuda-host-only; strict {} -x hip --offload-arch=gfx950 --cuda-host-only'
} | grep -v "^/opt/rocm" | sort -u > "$REPORT"

n=$(wc -l < "$REPORT")
echo "lint: $n finding(s) in $(echo $CPP $HIP | wc -w) files -> $REPORT"
[ "$n" -eq 0 ]
