#!/bin/bash
# Round 4: pass-B hashing probes (tools/probe_build.py), interleaved same-process timing
set -o pipefail
P=k2hash_amd/lib/probe
timeout -k 10 300 python3 tools/import_step.py --ab $P/nomiss.so,$P/nostore.so,$P/noslot.so,$P/nohash.so --no-parity --rounds 7 --calls 10 2>&1 | grep -v Warn
echo R04D_OK
