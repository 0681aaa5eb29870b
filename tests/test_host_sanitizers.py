"""The native host code of libolpe.so under AddressSanitizer + UndefinedBehaviorSanitizer
(CPU only: GPU sanitizers are not available on the pool, so the kernels are covered by
the parity tests and tests/test_kernel_resources.py instead).

olpe_csv.cpp -- the chain-file writer (repr-exact formatting, one file per walker from
a pool of threads, append mode for the streamed CLI) and the step-3 reader (block-wise
threaded parser) -- is built with g++
-fsanitize=address,undefined into a small driver and run over edge values (signed zero,
subnormals, the largest double, the repr fixed/scientific boundaries, non-finite values)
and a threaded write + append of many files.  Any sanitizer report aborts the driver;
its output must equal Python's repr / csv.writer bytes."""
import math
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "olpefit_amd", "csrc")

DRIVER = r"""
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "olpe.h"
namespace olpe {
int set_err(int code, const char *, ...) { return code; }   // (libolpe's lives in olpe.hip)
}
// fmt <hex doubles...>: one row, formatted with a NaN row first
// files <dir> <nfiles> <nrows> <ncols> <threads>: write (NaN row + rows), append rows,
//   values from a fixed LCG bit pattern, sizes printed
// read <dir> <nfiles> <nrows> <ncols> <threads>: write, then read back through the
//   step-3 reader (olpe_csv_read_chains) and compare the bits
static double bits(unsigned long long u) { double d; __builtin_memcpy(&d, &u, 8); return d; }
int main(int argc, char **argv) {
  const std::string mode = argv[1];
  if (mode == "fmt") {
    std::vector<double> v;
    for (int i = 2; i < argc; ++i) v.push_back(bits(strtoull(argv[i], nullptr, 16)));
    size_t len = 0;
    if (olpe_csv_format(v.data(), 1, (int)v.size(), 1, nullptr, 0, &len)) return 2;
    std::string s(len, '\0');
    if (olpe_csv_format(v.data(), 1, (int)v.size(), 1, &s[0], len, &len)) return 3;
    fwrite(s.data(), 1, len, stdout);
    return 0;
  }
  if (mode == "acc") {        // acc <dir> <nfiles> <np> <threads>: acceptance files
    const std::string dir = argv[2];
    const int nf = atoi(argv[3]), np_ = atoi(argv[4]), th = atoi(argv[5]);
    std::vector<std::string> names;
    std::vector<const char *> paths;
    for (int i = 0; i < nf; ++i) names.push_back(dir + "/" + std::to_string(i) + "_acc.csv");
    for (auto &n : names) paths.push_back(n.c_str());
    std::vector<double> acc((size_t)nf * np_), tries((size_t)nf * np_);
    unsigned long long x = 2463534242ull;
    for (size_t k = 0; k < acc.size(); ++k) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      tries[k] = (double)(1 + (x >> 40) % 100000);
      acc[k] = (double)((x >> 20) % (unsigned long long)tries[k]);
    }
    if (nf > 2) tries[np_] = acc[np_] = 0.0;            // row 1: NaN, left to the caller
    std::vector<unsigned char> done(nf, 9);
    if (olpe_acceptance_write(paths.data(), acc.data(), tries.data(), nf, np_, th, done.data()))
      return 12;
    for (int i = 0; i < nf; ++i) printf("%d\n", (int)done[i]);
    return 0;
  }
  const std::string dir = argv[2];
  const int nf = atoi(argv[3]), nr = atoi(argv[4]), nc = atoi(argv[5]), th = atoi(argv[6]);
  std::vector<std::string> names;
  std::vector<const char *> paths;
  for (int i = 0; i < nf; ++i) names.push_back(dir + "/" + std::to_string(i) + ".csv");
  for (auto &n : names) paths.push_back(n.c_str());
  std::vector<double> ch((size_t)nf * nr * nc);
  unsigned long long x = 88172645463325252ull;
  for (auto &d : ch) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    d = bits((x >> 2) | 0x3000000000000000ull) * ((x & 1) ? -1.0 : 1.0);
  }
  if (olpe_csv_write_chains(paths.data(), ch.data(), nf, nr, nc, 1, th)) return 4;
  if (mode == "read") {       // step 3's read of the same files, compared bit for bit
    long long rows = 0;
    int cols = 0;
    if (olpe_csv_shape(paths[0], &rows, &cols) || rows != nr + 1 || cols != nc) return 7;
    std::vector<double> back((size_t)nr * nf * nc);
    if (olpe_csv_read_chains(paths.data(), nf, rows, cols, 1, back.data(), th)) return 8;
    for (int i = 0; i < nf; ++i)
      for (int r = 0; r < nr; ++r)
        for (int c = 0; c < nc; ++c)
          if (__builtin_memcmp(&back[((size_t)r * nf + i) * nc + c],
                               &ch[((size_t)i * nr + r) * nc + c], 8))
            return 9;
    // a file with one row too many is an error naming it, not a crash
    if (olpe_csv_append_chains(paths.data(), ch.data(), 1, nr, 1, nc, 1, nullptr)) return 10;
    if (olpe_csv_read_chains(paths.data(), nf, rows, cols, 1, back.data(), th) != OLPE_EINVAL)
      return 11;
    printf("read ok\n");
    return 0;
  }
  std::vector<long long> sz(nf);
  if (olpe_csv_append_chains(paths.data(), ch.data(), nf, nr, nr / 2, nc, th, sz.data())) return 5;
  for (int i = 0; i < nf; ++i) printf("%lld\n", sz[i]);
  if (olpe_csv_append_chains(paths.data(), nullptr, 0, 0, 0, nc, th, nullptr)) return 6;
  return 0;
}
"""


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("san")
    src = d / "driver.cpp"
    src.write_text(DRIVER)
    exe = d / "driver"
    cmd = [gxx, "-g", "-O1", "-std=c++17", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", "-I" + os.path.join(REPO, "include"), "-o", str(exe),
           str(src), os.path.join(CSRC, "olpe_csv.cpp"), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "hip_runtime.h" in r.stderr:
        pytest.skip("HIP headers not available for a host-only build")
    assert r.returncode == 0, r.stderr
    return str(exe)


def _run(exe, *args):
    # (verify_asan_link_order=0: the environment may preload a library ahead of the
    # sanitizer runtime; nothing the driver calls is intercepted by it)
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, *args], capture_output=True, env=env, timeout=120)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0, err[-4000:]
    assert "runtime error" not in err and "AddressSanitizer" not in err, err
    return r.stdout.decode()            # bytes as written ("\r\n" kept)


def _hex(v):
    return "%016x" % struct.unpack("<Q", struct.pack("<d", v))[0]


def _repr(v):
    return "nan" if math.isnan(v) else repr(float(v))


def test_formatter_edge_values_under_sanitizers(driver):
    tiny = np.nextafter(0.0, 1.0)
    vals = [0.0, -0.0, tiny, -tiny, 2.2250738585072014e-308, 1.7976931348623157e308,
            -1.7976931348623157e308, 1e-5, 1e-4, 0.0001234, 9.999999999999999e-5,
            1e15, 9999999999999998.0, 1e16, 1.5e16, 123456789.125, 0.30000000000000004,
            -2.5, 1.0, 100.0, 1e22, 1e-300, float("nan"), float("inf"), float("-inf")]
    rng = np.random.default_rng(7)
    raw = rng.integers(0, 2 ** 64, size=200, dtype=np.uint64).view(np.float64)
    vals += [float(v) for v in raw]
    out = _run(driver, "fmt", *[_hex(v) for v in vals])
    nan_row, row, tail = out.split("\r\n")
    assert tail == "" and nan_row == ",".join(["nan"] * len(vals))
    assert row.split(",") == [_repr(v) for v in vals]


def test_threaded_write_and_append_under_sanitizers(driver, tmp_path):
    nf, nr, nc = 37, 12, 17
    sizes = [int(s) for s in _run(driver, "files", str(tmp_path), str(nf), str(nr), str(nc),
                                  "5").split()]
    assert len(sizes) == nf
    for i in range(nf):
        data = (tmp_path / f"{i}.csv").read_bytes()
        assert len(data) == sizes[i]
        lines = data.decode().split("\r\n")
        assert lines[-1] == "" and lines[0] == ",".join(["nan"] * nc)
        body = lines[1:-1]
        assert len(body) == nr + nr // 2 and body[nr:] == body[:nr // 2]
        assert all(len(l.split(",")) == nc for l in body)


@pytest.mark.parametrize("nf,nr", [(9, 40), (2, 20000)])
def test_threaded_reader_under_sanitizers(driver, tmp_path, nf, nr):
    """The reader parses in 4 MiB blocks: 2 x 20,000-row files (~8 MB each) carry lines
    across block ends; values come back bit for bit, a file of another length is an error."""
    assert _run(driver, "read", str(tmp_path), str(nf), str(nr), "17", "3").strip() == "read ok"


def test_acceptance_writer_under_sanitizers(driver, tmp_path):
    """olpe_acceptance_write from 5 threads: every fixed-notation row written (NumPy's
    str() of the same ratios, byte for byte), the NaN row left to the caller."""
    nf, npar = 23, 16
    done = [int(v) for v in _run(driver, "acc", str(tmp_path), str(nf), str(npar), "5").split()]
    assert done[1] == 0 and sum(done) == nf - 1
    x = 2463534242
    acc, tries = np.zeros(nf * npar), np.zeros(nf * npar)
    for k in range(nf * npar):
        x = (x * 6364136223846793005 + 1442695040888963407) % 2 ** 64
        tries[k] = 1 + (x >> 40) % 100000
        acc[k] = (x >> 20) % int(tries[k])
    for i in range(nf):
        if done[i]:
            want = str(acc[i * npar:(i + 1) * npar] / tries[i * npar:(i + 1) * npar])
            assert (tmp_path / f"{i}_acc.csv").read_text() == want


# -- ThreadSanitizer: the writer / reader thread pools (round 4, race detection) --------
@pytest.fixture(scope="module")
def tsan_driver(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("tsan")
    src = d / "driver.cpp"
    src.write_text(DRIVER)
    exe = d / "driver"
    cmd = [gxx, "-g", "-O1", "-std=c++17", "-fsanitize=thread", "-fno-omit-frame-pointer",
           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I" + os.path.join(REPO, "include"),
           "-o", str(exe), str(src), os.path.join(CSRC, "olpe_csv.cpp"), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "hip_runtime.h" in r.stderr:
        pytest.skip("HIP headers not available for a host-only build")
    assert r.returncode == 0, r.stderr
    return str(exe)


def _run_tsan(exe, *args):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([exe, *args], capture_output=True, env=env, timeout=300)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0, err[-4000:]
    assert "ThreadSanitizer" not in err, err[-4000:]
    return r.stdout.decode()


@pytest.mark.parametrize("mode", ["files", "read", "acc"])
def test_thread_pools_race_free(tsan_driver, tmp_path, mode):
    """The same driver under ThreadSanitizer: the threaded chain writer + append, the
    block-parallel step-3 reader and the acceptance writer, each from 6 threads, report
    no data race (the reference's host side is single-threaded per MPI rank; this
    build's file writers and reader are not)."""
    if mode == "acc":
        out = _run_tsan(tsan_driver, "acc", str(tmp_path), "31", "16", "6")
        assert len(out.split()) == 31
    elif mode == "read":
        assert _run_tsan(tsan_driver, "read", str(tmp_path), "3", "20000", "17",
                         "6").strip() == "read ok"
    else:
        assert len(_run_tsan(tsan_driver, "files", str(tmp_path), "29", "40", "17",
                             "6").split()) == 29
