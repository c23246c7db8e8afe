#!/bin/bash
# Microbenchmarks backing DESIGN.md §4 (VALU issue cost per instruction, SHA-256 variants).
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/valu_ubench > gpurun_out/valu_ubench.txt 2>&1 || exit $?
timeout -k 10 180 ./tools/sha_ubench > gpurun_out/sha_ubench.txt 2>&1 || exit $?
echo "ubench ok"
