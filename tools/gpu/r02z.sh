#!/bin/bash
# host-path chunk-size sweep (lab library, K2H_AMD_CHUNK_MB)
set -e
cd $GRAFT_REPO_ROOT
export K2H_AMD_BATCH_LIB=$GRAFT_REPO_ROOT/tools/lab/libk2hash_amd_lab.so
for mb in 64 16 32 128 64; do
  echo "chunk ${mb} MiB fixed:"; K2H_AMD_CHUNK_MB=$mb timeout -k 10 120 python -u tools/host_trace.py --reps 6 | tail -3
done
for mb in 64 32 128; do
  echo "chunk ${mb} MiB csr:"; K2H_AMD_CHUNK_MB=$mb timeout -k 10 120 python -u tools/host_trace.py --csr --n 8388608 --reps 5 | tail -2
done
