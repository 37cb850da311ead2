// Lab translation unit: the product CSR / long-key sources plus this round's experiments
// (one TU, so the product's non-inline functions are defined once).  Earlier rounds' lab
// sources are in git history (tools/lab/README.md).
#include "k2h_csr.hip"

#include "lab_fnv_y.inc"

#include "lab_csr_clock.inc"
#include "lab_csr_setup.inc"
#include "lab_csr_entry.inc"
