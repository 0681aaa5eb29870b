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
//
// The reader is step 3's side of the same files (apf_step3.py:169-186: one
// np.genfromtxt(..., delimiter=',') per walker file, collated into [rows, walkers]
// arrays): it parses every file from a pool of threads straight into that layout.
// std::from_chars rounds correctly, as Python's float() does, so the values are the
// ones genfromtxt returns, bit for bit.
#include <algorithm>
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

// --- reader (apf_step3.py:169-186) -------------------------------------------------
namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// one field as np.genfromtxt's float converter reads it: surrounding blanks stripped, an
// empty field is missing (NaN), 'nan' / 'inf' / '-inf' and a leading '+' accepted
bool parse_field(const char *a, const char *b, double &v) {
  while (a < b && is_space(*a)) ++a;
  while (b > a && is_space(b[-1])) --b;
  if (a == b) {
    v = std::nan("");
    return true;
  }
  if (*a == '+') ++a;
  const std::from_chars_result r = std::from_chars(a, b, v);
  return r.ec == std::errc() && r.ptr == b;
}

bool blank(const char *a, const char *b) {
  while (a < b && is_space(*a)) ++a;
  return a == b;
}

// The lines of a file (without the terminator), read in blocks of 4 MiB so that a long
// chain file (the reference's accept_min run records ~1.6 M rows, ~0.5 GB) never sits
// in memory whole; blank lines are skipped, as genfromtxt does.  Returns 1 when every
// line was handed to fn, 0 when fn stopped, -1 on a read error.
template <class F> int for_file_lines(const char *path, F &&fn) {
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  constexpr size_t kBlock = (size_t)1 << 22;
  std::vector<char> buf;
  size_t have = 0;             // a partial line carried over from the previous block
  int rc = 1;
  for (;;) {
    if (buf.size() < have + kBlock) buf.resize(have + kBlock);
    const size_t got = fread(buf.data() + have, 1, kBlock, f);
    if (got < kBlock && ferror(f)) {
      rc = -1;
      break;
    }
    const bool eof = got < kBlock;
    const char *p = buf.data(), *end = p + have + got;
    bool stop = false;
    for (;;) {
      const char *eol = (const char *)memchr(p, '\n', (size_t)(end - p));
      if (!eol) break;
      if (!blank(p, eol) && !fn(p, eol)) {
        stop = true;
        break;
      }
      p = eol + 1;
    }
    if (stop) {
      rc = 0;
      break;
    }
    if (eof) {                 // a last line without a terminator
      if (p < end && !blank(p, end) && !fn(p, end)) rc = 0;
      break;
    }
    have = (size_t)(end - p);
    memmove(buf.data(), p, have);
  }
  fclose(f);
  return rc;
}

}  // namespace

extern "C" {

int olpe_csv_shape(const char *path, long long *rows, int *cols) {
  if (!path || !rows || !cols) return olpe::set_err(OLPE_EINVAL, "olpe_csv_shape: NULL argument");
  long long n = 0;
  int c = 0;
  const int rc = for_file_lines(path, [&](const char *a, const char *b) {
    if (n++ == 0) {
      c = 1;
      for (const char *q = a; q < b; ++q) c += *q == ',';
    }
    return true;
  });
  if (rc < 0) return olpe::set_err(OLPE_EIO, "olpe_csv_shape: cannot read %s", path);
  *rows = n;
  *cols = c;
  return OLPE_OK;
}

int olpe_csv_read_chains(const char *const *paths, int nfiles, long long nrows, int ncols,
                         long long skip, double *out, int threads) {
  if (!paths || nfiles < 0 || nrows < 0 || ncols <= 0 || skip < 0 || skip > nrows ||
      (!out && nfiles > 0 && nrows > skip))
    return olpe::set_err(OLPE_EINVAL, "olpe_csv_read_chains: bad arguments");
  for (int i = 0; i < nfiles; ++i)
    if (!paths[i]) return olpe::set_err(OLPE_EINVAL, "olpe_csv_read_chains: path %d is NULL", i);
  unsigned nt = threads > 0 ? (unsigned)threads : std::thread::hardware_concurrency();
  if (nt == 0) nt = 1;
  if (nt > 64) nt = 64;
  if (nt > (unsigned)nfiles) nt = (unsigned)(nfiles > 0 ? nfiles : 1);
  // per thread: the first failing file and what went wrong
  std::vector<int> failed(nt, -1);
  std::vector<std::string> why(nt);
  auto work = [&](unsigned t) {
    char msg[160];
    for (int i = (int)t; i < nfiles; i += (int)nt) {
      long long row = 0;
      const int frc = for_file_lines(paths[i], [&](const char *a, const char *b) {
        if (row >= nrows) {
          snprintf(msg, sizeof(msg), "more than %lld rows (walker 0's length)", nrows);
          return false;
        }
        double *dst = out ? out + ((size_t)(row - skip) * (size_t)nfiles + (size_t)i) * (size_t)ncols
                          : nullptr;
        int col = 0;
        const char *f = a;
        for (;;) {
          const char *comma = (const char *)memchr(f, ',', (size_t)(b - f));
          const char *fe = comma ? comma : b;
          double v;
          if (col >= ncols) {
            snprintf(msg, sizeof(msg), "row %lld has more than %d fields", row, ncols);
            return false;
          }
          if (!parse_field(f, fe, v)) {
            snprintf(msg, sizeof(msg), "row %lld field %d is not a number", row, col);
            return false;
          }
          if (row >= skip) dst[col] = v;
          ++col;
          if (!comma) break;
          f = comma + 1;
        }
        if (col != ncols) {
          snprintf(msg, sizeof(msg), "row %lld has %d fields, not %d", row, col, ncols);
          return false;
        }
        ++row;
        return true;
      });
      if (frc < 0) {
        failed[t] = i;
        why[t] = "cannot read";
        return;
      }
      if (frc > 0 && row != nrows) snprintf(msg, sizeof(msg), "%lld rows, not %lld", row, nrows);
      if (frc == 0 || row != nrows) {
        failed[t] = i;
        why[t] = msg;
        return;
      }
    }
  };
  std::vector<std::thread> pool;
  for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto &th : pool) th.join();
  for (unsigned t = 0; t < nt; ++t)
    if (failed[t] >= 0)
      return olpe::set_err(why[t] == "cannot read" ? OLPE_EIO : OLPE_EINVAL,
                           "olpe_csv_read_chains: %s: %s", paths[failed[t]], why[t].c_str());
  return OLPE_OK;
}

}  // extern "C"

// --- acceptance files (apf_step2.py:362-365) -----------------------------------------
// The reference writes str(total_accept / total_tries): NumPy's print of a float64
// array.  For the arrays an accept / tries ratio gives -- every value finite, the
// non-zero ones in [1e-4, 1e8) and within a factor 1000 of each other -- NumPy prints
// in fixed notation ('maxprec', precision 8): each value's shortest round-trip digits,
// cut to 8 fractional digits (correctly rounded, trailing zeros dropped) when they are
// longer, the integer parts right-aligned and the fractions left-aligned to the widest,
// ' ' between values, '[' ... ']' and lines wrapped at 75 characters with a one-space
// indent (numpy/_core/arrayprint.py: FloatingFormat, _formatArray, _extendLine).  Other
// arrays (scientific notation, NaN from a never-tried parameter) are left to the caller.
namespace {

// digits of v >= 0 as NumPy's dragon4_positional(v, precision=8, unique=True,
// fractional=True, trim='.'): integer part and fraction (without the point)
void positional8(double v, std::string &ip, std::string &fp) {
  char buf[64];
  std::to_chars_result r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::fixed);
  std::string s(buf, r.ptr);
  size_t dot = s.find('.');
  if (dot != std::string::npos && s.size() - dot - 1 > 8) {
    r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::fixed, 8);
    s.assign(buf, r.ptr);
    dot = s.find('.');
    while (!s.empty() && s.back() == '0') s.pop_back();
  }
  if (dot == std::string::npos) {
    ip = s;
    fp.clear();
  } else {
    ip = s.substr(0, dot);
    fp = s.substr(dot + 1);
  }
}

// str(np.array(x)) for x[0..n) in the fixed-notation range; false otherwise
bool numpy_str_fixed(const double *x, int n, std::string &out) {
  double mx = 0.0, mn = 0.0;
  bool any = false;
  for (int i = 0; i < n; ++i) {
    if (!std::isfinite(x[i]) || x[i] < 0.0 || std::signbit(x[i])) return false;
    if (x[i] != 0.0) {
      mx = any ? std::max(mx, x[i]) : x[i];
      mn = any ? std::min(mn, x[i]) : x[i];
      any = true;
    }
  }
  if (any && (mx >= 1.e8 || mn < 0.0001 || mx / mn > 1000.)) return false;
  std::vector<std::string> ip(n), fp(n);
  size_t pl = 0, pr = 0;
  for (int i = 0; i < n; ++i) {
    positional8(x[i], ip[i], fp[i]);
    pl = std::max(pl, ip[i].size());
    pr = std::max(pr, fp[i].size());
  }
  // _formatArray, one axis: line width 75 - len(']'), hanging indent ' '
  const size_t width = 74;
  std::string s, line = " ";
  for (int i = 0; i < n; ++i) {
    std::string word(pl - ip[i].size(), ' ');
    word += ip[i];
    word += '.';
    word += fp[i];
    word.append(pr - fp[i].size(), ' ');
    if (line.size() + word.size() > width && line.size() > 1) {
      size_t e = line.find_last_not_of(' ');
      s.append(line, 0, e == std::string::npos ? 0 : e + 1);
      s += '\n';
      line = " ";
    }
    line += word;
    if (i + 1 < n) line += ' ';
  }
  s += line;
  out = "[" + s.substr(1) + "]";
  return true;
}

}  // namespace

extern "C" {

int olpe_acceptance_format(const double *x, int n, char *out, size_t cap, size_t *len_out) {
  if (!x || n <= 0 || !len_out) return olpe::set_err(OLPE_EINVAL, "olpe_acceptance_format: bad arguments");
  std::string s;
  if (!numpy_str_fixed(x, n, s)) {
    *len_out = 0;
    return OLPE_OK;
  }
  *len_out = s.size();
  if (out) {
    if (cap < s.size()) return olpe::set_err(OLPE_EINVAL, "olpe_acceptance_format: %zu bytes needed", s.size());
    memcpy(out, s.data(), s.size());
  }
  return OLPE_OK;
}

int olpe_acceptance_write(const char *const *paths, const double *accepts, const double *tries,
                          int nfiles, int np, int threads, unsigned char *done) {
  if (!paths || !accepts || !tries || !done || nfiles < 0 || np <= 0)
    return olpe::set_err(OLPE_EINVAL, "olpe_acceptance_write: bad arguments");
  unsigned nt = threads > 0 ? (unsigned)threads : std::thread::hardware_concurrency();
  if (nt == 0) nt = 1;
  if (nt > 64) nt = 64;
  if (nt > (unsigned)nfiles) nt = (unsigned)(nfiles > 0 ? nfiles : 1);
  std::vector<int> failed(nt, -1);
  auto work = [&](unsigned t) {
    std::vector<double> x(np);
    std::string s, tmp;
    for (int i = (int)t; i < nfiles; i += (int)nt) {
      for (int k = 0; k < np; ++k) x[k] = accepts[(size_t)i * np + k] / tries[(size_t)i * np + k];
      done[i] = 0;
      if (!paths[i] || !numpy_str_fixed(x.data(), np, s)) continue;
      // a temporary name renamed over the file: a run killed mid-write leaves the
      // previous complete file, never a truncated one (the checkpoint's acceptance
      // files are written in the background)
      tmp.assign(paths[i]).append(".tmp");
      // every failure removes the temporary file (no '<path>.tmp' left behind)
      FILE *f = fopen(tmp.c_str(), "wb");
      if (!f || fwrite(s.data(), 1, s.size(), f) != s.size()) {
        if (f) fclose(f);
        (void)remove(tmp.c_str());
        failed[t] = i;
        return;
      }
      if (fclose(f) != 0 || rename(tmp.c_str(), paths[i]) != 0) {
        (void)remove(tmp.c_str());
        failed[t] = i;
        return;
      }
      done[i] = 1;
    }
  };
  std::vector<std::thread> pool;
  for (unsigned t = 1; t < nt; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto &th : pool) th.join();
  for (unsigned t = 0; t < nt; ++t)
    if (failed[t] >= 0)
      return olpe::set_err(OLPE_EIO, "olpe_acceptance_write: cannot write %s", paths[failed[t]]);
  return OLPE_OK;
}

}  // extern "C"
