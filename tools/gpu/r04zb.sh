#!/bin/bash
# Round 4 final (after the import / RALLEDATA work of the second half): the GPU suite, the
# default bench line, the round profile of every bench config and the k2himport profile;
# then a RALLEDATA A/B of the staging loop's stream selection by selects (probe/ralsel.so).
set -o pipefail
TAG=r04zb bash tools/gpu/r04z.sh || exit 1
timeout -k 10 300 python3 tools/ab_libs.py --config ralledata --libs k2hash_amd/lib/probe/ralsel.so 2>&1 | grep -v Warn | cut -c1-160
