"""CPU checks of the C-ABI library: it loads, exports every symbol include/olpe.h
declares, the ctypes signatures match the header, and calls fail cleanly (no abort)
on a host without a GPU.  No compute calls."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from olpefit_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "olpe.h")
# the test hooks: exported, declared apart from the stable C-ABI
TEST_HEADER = os.path.join(REPO, "include", "olpe_test.h")


def header_functions(paths=(HEADER, TEST_HEADER)):
    names = set()
    for p in paths:
        text = re.sub(r"/\*.*?\*/", "", open(p).read(), flags=re.S)
        names |= set(re.findall(r"\b(olpe_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    from olpefit_amd import build
    build.build(verbose=False)
    return _lib.load()


def test_header_declares_expected_api():
    names = header_functions((HEADER,))
    for must in ("olpe_create", "olpe_model", "olpe_chi2_batch", "olpe_seed", "olpe_run",
                 "olpe_run_gibbs", "olpe_rng_get", "olpe_rng_set", "olpe_destroy",
                 "olpe_last_error", "olpe_comm_allgather_state", "olpe_comm_info",
                 "olpe_comm_timeout"):
        assert must in names
    # the fault hooks are not part of the stable C-ABI: only the test header has them
    assert "olpe_moments_fault" not in names
    assert "olpe_moments_fault" in header_functions((TEST_HEADER,))


def test_library_exports_every_header_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s+(olpe_\w+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing
    # ctypes table covers the header one-to-one
    assert sorted(_lib.SIGNATURES) == header_functions()


def test_version_and_device_count(lib):
    assert lib.olpe_version() >= 100
    n = C.c_int(-1)
    assert lib.olpe_device_count(C.byref(n)) == 0
    assert n.value >= 0


def test_create_validates_arguments_before_touching_a_gpu(lib):
    img = np.zeros((8, 9), np.float32)
    ctx = C.c_void_p()
    rc = lib.olpe_create(img.ctypes.data, 0, img.ctypes.data, 1444.0, None, 8, 9, 2, 0, 0,
                         C.byref(ctx))
    assert rc == _lib.EINVAL and b"square" in lib.olpe_last_error()
    img = np.zeros((8, 8), np.float32)
    assert lib.olpe_create(img.ctypes.data, 0, img.ctypes.data, 1444.0, None, 8, 8, 4, 0, 0,
                           C.byref(ctx)) == _lib.EINVAL
    assert lib.olpe_create(img.ctypes.data, 0, img.ctypes.data, 1444.0, None, 8, 8, 2, 0, -1,
                           C.byref(ctx)) == _lib.EINVAL          # no CPU path


def test_no_gpu_fails_loudly(lib):
    n = C.c_int(0)
    lib.olpe_device_count(C.byref(n))
    if n.value:
        pytest.skip("GPU present")
    from olpefit_amd.core import OlpeError, Sampler
    with pytest.raises(OlpeError) as e:
        Sampler(np.ones((16, 16), np.float32))
    assert e.value.code == _lib.EHIP


def test_null_arguments_are_errors(lib):
    assert lib.olpe_model(None, None, None) == _lib.EINVAL
    assert lib.olpe_run(None, 1, 0, 1, 0, None) == _lib.EINVAL
    assert lib.olpe_sync(None) == _lib.EINVAL
    assert lib.olpe_moments_accumulate(None) == _lib.EINVAL
    assert lib.olpe_moments_reset(None) == _lib.EINVAL
    assert lib.olpe_moments_get(None, None, None, None) == _lib.EINVAL
    assert lib.olpe_moments_set(None, 0, None, None) == _lib.EINVAL
    assert lib.olpe_moments_summary(None, None, None) == _lib.EINVAL
    assert lib.olpe_comm_allreduce_moments(None, None) == _lib.EINVAL
    assert lib.olpe_csv_shape(None, None, None) == _lib.EINVAL
    assert lib.olpe_csv_read_chains(None, 1, 1, 1, 0, None, 0) == _lib.EINVAL
    lib.olpe_destroy(None)


def test_empty_and_oversized_cutouts_are_rejected(lib):
    """Shapes the reference cannot take either: an empty image, one wider than the
    4096-pixel limit, an unknown dtype, a NULL image -- EINVAL before any GPU call."""
    ctx = C.c_void_p()
    img = np.zeros((8, 8), np.float32)
    for ny, nx, dt, ptr in ((0, 0, 0, img.ctypes.data), (4097, 4097, 0, img.ctypes.data),
                            (8, 8, 7, img.ctypes.data), (8, 8, 0, None)):
        assert lib.olpe_create(ptr, dt, img.ctypes.data, 1444.0, None, ny, nx, 2, 0, 0,
                               C.byref(ctx)) == _lib.EINVAL, (ny, nx, dt)
    assert not ctx.value
    # a side whose one-wave row tables exceed the LDS (3 sources, 48 B per row)
    assert lib.olpe_create(img.ctypes.data, 0, img.ctypes.data, 1444.0, None, 4000, 4000, 3,
                           0, 0, C.byref(ctx)) == _lib.EINVAL
    assert b"LDS" in lib.olpe_last_error()


def test_wpb_knob_is_validated_against_the_lds(lib, monkeypatch):
    """OLPE_WPB (a tuning knob) is checked in olpe_create against the 160 KiB LDS before
    anything touches a GPU: 16 waves of the 3-source 64x64 sampler do not fit beside the
    cutout, so the launch would fail (the 2-source FAST one does, with its single
    shape-table slot); 7 is not a workgroup size."""
    img = np.ones((64, 64), np.float32)
    ctx = C.c_void_p()

    def create(nsrc=2):
        return lib.olpe_create(img.ctypes.data, 0, img.ctypes.data, 1444.0, None, 64, 64, nsrc,
                               0, 0, C.byref(ctx))
    monkeypatch.setenv("OLPE_WPB", "16")
    assert create(nsrc=3) == _lib.EINVAL
    msg = lib.olpe_last_error().decode()
    assert "bytes of LDS" in msg and int(re.search(r"needs (\d+) bytes", msg).group(1)) > 163840
    monkeypatch.setenv("OLPE_WPB", "7")
    assert create() == _lib.EINVAL and b"8, 12 or 16" in lib.olpe_last_error()
    n = C.c_int(0)
    lib.olpe_device_count(C.byref(n))
    for wpb in ("12", "16"):
        monkeypatch.setenv("OLPE_WPB", wpb)
        if not n.value:
            assert create() == _lib.EHIP        # valid knob: fails only for lack of a GPU


def test_kernel_digest_covers_only_the_sampler_bundle():
    """The VALU counts in profiles/ are tagged with the hash of the sampler's code-object
    bundle only: another source's kernels (olpe_moments.hip) may change without marking
    them stale, a change inside the sampler's bundle does; the built library's digest is
    the one its section gives."""
    from olpefit_amd.build import fatbin_digest, kernel_digest, _elf_section, LIB
    m = b"__CLANG_OFFLOAD_BUNDLE__"
    a = m + b"..olpe_gibbs_kernel..code-A.."
    b = m + b"..fold_kernel..code-B.."
    ref = fatbin_digest(a + b)
    assert fatbin_digest(a + m + b"..fold_kernel..code-B2..") == ref
    assert fatbin_digest(m + b"..olpe_gibbs_kernel..code-A2.." + b) != ref
    assert fatbin_digest(b"no bundles") != ref
    if os.path.exists(LIB):
        assert kernel_digest() == fatbin_digest(_elf_section(LIB, ".hip_fatbin"))


def _elf(sections):
    """A minimal ELF64 little-endian image with the given {name: bytes} sections."""
    import struct
    names = [""] + list(sections) + [".shstrtab"]
    strtab, offs = b"", []
    for n in names:
        offs.append(len(strtab))
        strtab += n.encode() + b"\0"
    body, places = b"", []
    for n in names[1:-1]:
        places.append((64 + len(body), len(sections[n])))
        body += sections[n]
    places.append((64 + len(body), len(strtab)))
    body += strtab
    shoff = 64 + len(body)
    hdr = bytearray(64)
    hdr[:6] = b"\x7fELF\x02\x01"
    struct.pack_into("<Q", hdr, 0x28, shoff)
    struct.pack_into("<HHH", hdr, 0x3A, 64, len(names), len(names) - 1)
    shdrs = bytes(64)
    for i, (off, size) in enumerate(places):
        shdrs += struct.pack("<IIQQQQ", offs[i + 1], 1, 0, 0, off, size) + bytes(24)
    return bytes(hdr) + body + shdrs


def test_kernel_digest_hashes_the_code_sections():
    """Within the sampler's bundle only the code object's code sections count: its
    symbol table (ordered by the per-build unit ids, __hip_cuid_*, which follow the
    compile command) may differ without changing the digest; its instructions may not."""
    from olpefit_amd.build import fatbin_digest
    m = b"__CLANG_OFFLOAD_BUNDLE__..olpe_gibbs_kernel.."
    code = {".text": b"\x01\x02\x03\x04" * 8, ".rodata": b"kd" * 8, ".note": b"meta"}
    a = _elf({**code, ".symtab": b"__hip_cuid_1111111111111111 olpe_gibbs_kernel"})
    b = _elf({".symtab": b"olpe_gibbs_kernel __hip_cuid_2222222222222222", **code})
    c = _elf({**code, ".text": b"\x01\x02\x03\x05" * 8, ".symtab": b"x"})
    assert fatbin_digest(m + a) == fatbin_digest(m + b"pad" + b)
    assert fatbin_digest(m + a) != fatbin_digest(m + c)


def test_comm_calls_without_a_communicator_fail_cleanly(lib):
    assert lib.olpe_comm_timeout(None, 1.0) == _lib.EINVAL
    n, r = C.c_int(0), C.c_int(0)
    assert lib.olpe_comm_info(None, C.byref(n), C.byref(r)) == _lib.EINVAL


def test_product_sources_carry_no_diagnostic_hooks():
    """Verdict r05 item 4: the diagnostic builds' hooks live in tools/diag/diag_hooks.patch,
    applied by tools/diag_build.sh to a copy of the sources; the product sources name
    none of them, and the patch still applies to them."""
    import shutil
    import tempfile
    csrc = os.path.join(REPO, "olpefit_amd", "csrc")
    for f in os.listdir(csrc):
        text = open(os.path.join(csrc, f)).read()
        assert not re.search(r"OLPE_(DIAG|EXP)_|DT_MARK|diag_fill_kernel|g_diag_fb", text), f
    if not shutil.which("patch"):
        pytest.skip("patch(1) not available")
    with tempfile.TemporaryDirectory() as td:
        shutil.copytree(csrc, os.path.join(td, "olpefit_amd", "csrc"))
        os.makedirs(os.path.join(td, "include"))
        shutil.copy(HEADER, os.path.join(td, "include"))
        r = subprocess.run(["patch", "-p1", "--dry-run", "-d", td, "-i",
                            os.path.join(REPO, "tools", "diag", "diag_hooks.patch")],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "FAILED" not in r.stdout and "fuzz" not in r.stdout, r.stdout


def test_proposal_widths_are_inside_the_digest(lib):
    """the __constant__ proposal widths (olpe.hip c_widths2 / c_widths3,
    apf_step2.py:234) sit in a section the kernel digest hashes, so editing one marks the
    measured counts stale: flipping a byte of them in the sampler's code object changes
    the digest."""
    import struct
    from olpefit_amd.build import CODE_SECTIONS, LIB, _elf_section, _elf_sections, fatbin_digest
    fat = _elf_section(LIB, ".hip_fatbin")
    assert fat
    pat = b"".join(struct.pack("<d", v) for v in (0.0025, 0.02, 0.001, 0.0008))
    start = fat.index(b"__CLANG_OFFLOAD_BUNDLE__")
    hits = [m.start() for m in re.finditer(re.escape(pat), fat)]
    assert hits, "widths not found in the fat binary"
    # the widths are in a code section of an ELF object of the sampler's bundle
    found = False
    i = fat.find(b"\x7fELF", start)
    while i >= 0:
        secs = _elf_sections(fat[i:])
        if any(pat in secs.get(n, b"") for n in CODE_SECTIONS):
            found = True
            break
        i = fat.find(b"\x7fELF", i + 4)
    assert found, "widths outside the digested sections"
    h = hits[0]
    mutated = fat[:h] + bytes([fat[h] ^ 1]) + fat[h + 1:]
    assert fatbin_digest(mutated) != fatbin_digest(fat)
