#!/bin/bash
# Host-code sanitizer run: builds the GraphDef codec fuzz
# harness with AddressSanitizer + UndefinedBehaviorSanitizer (host only, no
# GPU code involved) and runs it over the fixture graphs.
#   scripts/sanitize_host.sh [ITERATIONS]
set -euo pipefail
cd "$(dirname "$0")/.."
ITERS=${1:-20000}
OUT=${TMPDIR:-/tmp}/tfa_proto_fuzz
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    -Icsrc csrc/tests/proto_fuzz.cpp csrc/proto/graphdef.cpp -o "$OUT"
TFA_MAX_CONST_BYTES=$((64 << 20)) ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
    "$OUT" "$ITERS" tests/fixtures/ref_graph.pb tests/fixtures/ref_graph2.pb tests/fixtures/*.pb
