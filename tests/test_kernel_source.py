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


@pytest.fixture(scope="module")
def import_asm(tmp_path_factory):
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm") / "k2h_import_dev.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                    f"-I{ROOT / 'include'}", str(CSRC / "k2h_import_dev.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    return out.read_text()


def _kernel_meta(asm: str):
    """{kernel symbol: its amdhsa metadata fields} from the assembly's metadata block."""
    meta = {}
    for block in re.split(r"\n\s+- \.agpr_count:", asm):
        m = re.search(r"\.name:\s+(_Z\w+)", block)
        if not m:
            continue
        fields = dict(re.findall(r"\.(\w+):\s+(\d+)\s*$", block, flags=re.M))
        meta[m.group(1)] = {k: int(v) for k, v in fields.items()}
    return meta


def test_import_kernels_use_no_scratch_and_keep_pass_a_occupancy(import_asm):
    """Round 4: a lambda in pass A's event walk once made hipcc keep two values in scratch
    (12 B per lane, stored inside the loop): pass A 318 -> 420 us.  Every import kernel
    must run without scratch or spills, and pass A's TSV block must stay within 35 LDS
    granules of 512 B (17,920 B: 9 blocks per CU; one granule more cost 11 %)."""
    meta = _kernel_meta(import_asm)
    kernels = {k: v for k, v in meta.items() if "tsv_" in k or "import_hash" in k}
    assert len(kernels) >= 6, sorted(meta)
    for sym, f in kernels.items():
        assert f.get("private_segment_fixed_size", 0) == 0, sym
        assert f.get("vgpr_spill_count", 0) == 0 and f.get("sgpr_spill_count", 0) == 0, sym
    pass_a = [v for k, v in kernels.items() if "tsv_a_kernelILb0" in k]
    assert len(pass_a) == 1
    assert pass_a[0]["group_segment_fixed_size"] <= 35 * 512
    assert pass_a[0]["vgpr_count"] <= 64  # 8 waves per SIMD's worth of registers; LDS sets 4.5
    # pass B: 59 VGPRs for the TSV prehash form since round 5 (8 waves per SIMD;
    # 68 had held it at 7): every instantiation stays within 64
    pass_b = {k: v for k, v in kernels.items() if "tsv_b_kernel" in k}
    assert len(pass_b) == 4, sorted(pass_b)
    for sym, f in pass_b.items():
        assert f["vgpr_count"] <= 64, (sym, f["vgpr_count"])


def test_import_file_reads_are_bounds_guarded():
    """Every device hash of a key read from the file goes through hash_cstr_checked, whose
    range check against the file size is the only caller of the unchecked body (ADVICE r4:
    pass B's miss path faulted on a probe's wrong states; ADVICE r5: a text check next to
    each call could be satisfied by an unrelated comparison).  A wrong state must give
    wrong records that parity catches, not a device fault."""
    text = (CSRC / "k2h_import_dev.hip").read_text()
    code = re.sub(r"//[^\n]*", "", text)  # comments out
    unchecked = [m.start() for m in re.finditer(r"\bhash_cstr_unchecked\s*\(", code)]
    assert len(unchecked) == 2, "the definition and the one call inside hash_cstr_checked"
    body = code[code.index("void hash_cstr_checked("):]
    body = body[:body.index("\n}\n")]
    assert "if (off <= size && len <= size - off)" in body and "hash_cstr_unchecked(" in body
    assert code.index("void hash_cstr_checked(") < unchecked[1] < code.index("void hash_cstr_checked(") + len(body)
    assert len(re.findall(r"\bhash_cstr_checked\s*\(f,\s*size,", code)) >= 3
    assert not re.search(r"\bhash_cstr\s*\(", code), "a file hash outside the checked wrapper"