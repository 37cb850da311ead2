"""Static checks of the product kernel sources and their gfx950 code (CPU only).

* The product sources carry no measurement-lab code (the round-2 A/B
  variants live in tools/lab/src/r02/, archived).
* Partial vmcnt waits are only correct under an ordering invariant: the line-DMA kernel
  waits with `s_waitcnt vmcnt(NP*(D-1))` for "round q has landed", which holds only if the
  wave issues no vector-memory store inside its round loop (stores would count in vmcnt
  and could retire out of order w.r.t. the DMA loads).  The disassembly is scanned: in
  every instantiation of fnv_fixed_lines_kernel, every global/buffer/flat store comes
  after the last LDS-DMA load.
"""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "k2hash_amd" / "csrc"
HIPCC = "/opt/rocm/bin/hipcc"


def test_product_sources_have_no_lab_sections():
    for f in sorted(CSRC.iterdir()):
        if f.suffix in (".hip", ".cc", ".h", ".inc"):
            text = f.read_text()
            assert "K2H_AMD_LAB" not in text, f.name
            assert "_lab.inc" not in text, f.name
    assert not list(CSRC.glob("*_lab*.inc"))


@pytest.fixture(scope="module")
def csr_asm(tmp_path_factory):
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm") / "k2h_csr.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                    str(CSRC / "k2h_csr.hip"), "-o", str(out)], check=True, capture_output=True)
    return out.read_text()


def _functions(asm: str, name_part: str):
    """(symbol, body) of every kernel whose mangled name contains name_part."""
    out = []
    for m in re.finditer(r"^(_Z\w*" + name_part + r"\w*):", asm, flags=re.M):
        end = asm.find(".Lfunc_end", m.end())
        out.append((m.group(1), asm[m.end():end]))
    return out


def test_lines_kernel_stores_follow_all_dma_loads(csr_asm):
    funcs = _functions(csr_asm, "fnv_fixed_lines_kernel")
    assert funcs, "fnv_fixed_lines_kernel not found in the disassembly"
    for sym, body in funcs:
        ins = [ln.strip() for ln in body.splitlines() if ln.strip() and not ln.strip().startswith((";", "."))]
        dma = [i for i, s in enumerate(ins) if re.match(r"global_load_lds|buffer_load_dword\w* .*lds", s)]
        stores = [i for i, s in enumerate(ins) if re.match(r"(global|buffer|flat)_store", s)]
        assert dma, sym
        assert stores, sym
        assert min(stores) > max(dma), f"{sym}: a vector store precedes the last LDS-DMA load"
        waits = [s for s in ins if s.startswith("s_waitcnt") and "vmcnt(" in s]
        assert any("vmcnt(8)" in s for s in waits), f"{sym}: expected the partial vmcnt(NP*(D-1)) wait"


def test_lines_kernel_has_no_compiler_m0_use(csr_asm):
    """The line-DMA kernel writes M0 inside its own asm DMA statements (line_dma8) without
    saving it.  That is only safe while hipcc itself never relies on M0 in the kernel: no
    instruction outside the asm statements may name m0."""
    funcs = _functions(csr_asm, "fnv_fixed_lines_kernel")
    assert funcs
    for sym, body in funcs:
        inside, hits = False, []
        for ln in body.splitlines():
            s = ln.strip()
            if s.startswith(";;#ASMSTART"):
                inside = True
            elif s.startswith(";;#ASMEND"):
                inside = False
            elif not inside and not s.startswith((";", ".")) and re.search(r"\bm0\b", s):
                hits.append(s)
        assert not hits, f"{sym}: compiler-emitted M0 use {hits[:3]}"
