// olpe_csv.cpp -- the chain file writer of apf_step2 (host code of libolpe.so).
//
// The reference appends every recorded state to `total_parameters` and rewrites
// `{rank}_finalarray_mpi.csv` with csv.writer(...).writerows(total_parameters)
// (apf_step2.py:342-360; 3body/apf_step2_3body.py:381-399).  csv.writer formats a
// float with repr(): the shortest digit string that reads back to the same double,
// in fixed notation when the decimal exponent X (value = d.ddd x 10^X) satisfies
// -4 <= X < 16 and in scientific notation otherwise ('1e-05', '1.5e+16'), a fixed
// value without a fractional part gets '.0', non-finite values are 'nan' / 'inf' /
// '-inf'; fields are joined by ',' and rows end in "\r\n".  This writer produces the
// same bytes (std::to_chars gives the shortest round-trip digits, like repr) and
// writes one file per walker from a pool of threads: at 10^5 walkers x 10^2 rows the
// Python formatter takes minutes, this one the time of the disk writes.
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/olpe.h"
#include "olpe_internal.h"

namespace {

// repr(float) of v, appended to out
void append_repr(std::string &out, double v) {
  if (std::isnan(v)) {
    out += "nan";
    return;
  }
  if (std::isinf(v)) {
    out += v < 0 ? "-inf" : "inf";
    return;
  }
  char buf[64];
  const std::to_chars_result r =
      std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  // buf = [-]d[.ddd]e(+|-)XX[X]
  const char *p = buf;
  const char *end = r.ptr;
  bool neg = false;
  if (*p == '-') {
    neg = true;
    ++p;
  }
  char digits[32];
  int nd = 0;
  const char *e = p;
  while (e < end && *e != 'e') {
    if (*e != '.') digits[nd++] = *e;
    ++e;
  }
  int x = 0;
  std::from_chars(e + 1 + (e[1] == '+' ? 1 : 0), end, x);
  if (neg) out += '-';
  if (x >= -4 && x < 16) {
    if (x < 0) {                                   // 0.000ddd
      out += "0.";
      out.append((size_t)(-x - 1), '0');
      out.append(digits, (size_t)nd);
    } else if (nd <= x + 1) {                      // ddd000.0
      out.append(digits, (size_t)nd);
      out.append((size_t)(x + 1 - nd), '0');
      out += ".0";
    } else {                                       // ddd.ddd
      out.append(digits, (size_t)(x + 1));
      out += '.';
      out.append(digits + x + 1, (size_t)(nd - x - 1));
    }
    return;
  }
  out += digits[0];
  if (nd > 1) {
    out += '.';
    out.append(digits + 1, (size_t)(nd - 1));
  }
  char ex[16];
  const int ax = x < 0 ? -x : x;
  snprintf(ex, sizeof(ex), "e%c%02d", x < 0 ? '-' : '+', ax);
  out += ex;
}

void format_rows(std::string &out, const double *rows, long long nrows, int ncols,
                 bool nan_row) {
  out.reserve(out.size() + (size_t)(nrows + 1) * (size_t)ncols * 20);
  if (nan_row) {
    for (int c = 0; c < ncols; ++c) {
      if (c) out += ',';
      out += "nan";
    }
    out += "\r\n";
  }
  for (long long i = 0; i < nrows; ++i) {
    const double *row = rows + i * ncols;
    for (int c = 0; c < ncols; ++c) {
      if (c) out += ',';
      append_repr(out, row[c]);
    }
    out += "\r\n";
  }
}

}  // namespace

extern "C" {

int olpe_csv_format(const double *rows, long long nrows, int ncols, int nan_row, char *out,
                    size_t cap, size_t *len_out) {
  if ((!rows && nrows > 0) || nrows < 0 || ncols <= 0 || !len_out)
    return olpe::set_err(OLPE_EINVAL, "olpe_csv_format: bad arguments");
  std::string s;
  format_rows(s, rows, nrows, ncols, nan_row != 0);
  *len_out = s.size();
  if (out) {
    if (cap < s.size())
      return olpe::set_err(OLPE_EINVAL, "olpe_csv_format: buffer of %zu bytes < %zu", cap,
                           s.size());
    memcpy(out, s.data(), s.size());
  }
  return OLPE_OK;
}

}  // extern "C"

namespace {

// Write (mode "wb") or append (mode "ab") file i <- rows [0, nrows) of
// chains[i][rows_per_file][ncols], from a pool of threads; sizes_out[i] = the file's
// size in bytes after the write (or NULL).
int write_files(const char *fn, const char *const *paths, const double *chains, int nfiles,
                long long rows_per_file, long long nrows, int ncols, bool nan_row, int threads,
                const char *mode, long long *sizes_out) {
  if (!paths || nfiles < 0 || nrows < 0 || rows_per_file < nrows || ncols <= 0 ||
      (!chains && nrows > 0 && nfiles > 0))
    return olpe::set_err(OLPE_EINVAL, "%s: bad arguments", fn);
  for (int i = 0; i < nfiles; ++i)
    if (!paths[i]) return olpe::set_err(OLPE_EINVAL, "%s: path %d is NULL", fn, i);
  unsigned nt = threads > 0 ? (unsigned)threads : std::thread::hardware_concurrency();
  if (nt == 0) nt = 1;
  if (nt > 64) nt = 64;
  if (nt > (unsigned)nfiles) nt = (unsigned)(nfiles > 0 ? nfiles : 1);
  std::vector<int> failed(nt, -1);
  auto work = [&](unsigned t) {
    std::string s;
    for (int i = (int)t; i < nfiles; i += (int)nt) {
      s.clear();
      format_rows(s, chains ? chains + (size_t)i * (size_t)rows_per_file * (size_t)ncols : nullptr,
                  nrows, ncols, nan_row);
      FILE *f = fopen(paths[i], mode);
      bool ok = f && fwrite(s.data(), 1, s.size(), f) == s.size();
      long long size = 0;
      if (ok && sizes_out) {
        ok = fflush(f) == 0 && fseek(f, 0, SEEK_END) == 0;
        size = ok ? (long long)ftell(f) : -1;
        ok = ok && size >= 0;
      }
      if (f && fclose(f) != 0) ok = false;
      if (!ok) {
        failed[t] = i;
        return;
      }
      if (sizes_out) sizes_out[i] = size;
    }
  };
  std::vector<std::thread> pool;
  for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto &th : pool) th.join();
  for (unsigned t = 0; t < nt; ++t)
    if (failed[t] >= 0) return olpe::set_err(OLPE_EIO, "%s: cannot write %s", fn, paths[failed[t]]);
  return OLPE_OK;
}

}  // namespace

extern "C" {

int olpe_csv_write_chains(const char *const *paths, const double *chains, int nfiles,
                          long long nrows, int ncols, int nan_row, int threads) {
  return write_files("olpe_csv_write_chains", paths, chains, nfiles, nrows, nrows, ncols,
                     nan_row != 0, threads, "wb", nullptr);
}

int olpe_csv_append_chains(const char *const *paths, const double *chains, int nfiles,
                           long long rows_per_file, long long nrows, int ncols, int threads,
                           long long *sizes_out) {
  return write_files("olpe_csv_append_chains", paths, chains, nfiles, rows_per_file, nrows,
                     ncols, false, threads, "ab", sizes_out);
}

}  // extern "C"
