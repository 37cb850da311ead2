#!/bin/bash
# Issue / wait PMC breakdown of the final CSR product kernel (lean2, variant 0) beside the
# queue kernel (87) and the dbuf kernel (81), one rocprofv3 --pmc run per counter group.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_csr_r02bh CONFIG=csr bash tools/pmc_variants.sh 0 87 81
python3 tools/pmc_table.py gpurun_out/pmc_csr_r02bh > gpurun_out/r02bh_pmc_csr.txt
cat gpurun_out/r02bh_pmc_csr.txt
