// Round-3 lab translation unit: the product CSR / long-key sources plus the experiments
// (one TU, so the product's non-inline functions are defined once).
#include "k2h_csr.hip"

#include "lab_lines.inc"
#include "lab_csr_setup.inc"
#include "lab_csr.inc"
#include "lab_csr_rs.inc"
#include "lab_csr_rs2.inc"
#include "lab_csr_rs4.inc"
#include "lab_csr_lean.inc"
