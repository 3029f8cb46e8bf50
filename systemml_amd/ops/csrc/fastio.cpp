// Multi-threaded text readers for the host IO path (reference analogue:
// runtime/io/ReaderTextCSVParallel.java and ReaderTextCellParallel.java, which split the
// input into line-aligned ranges and parse them with a thread pool).
//
// The file is memory-mapped; [0, size) is cut into `threads` byte ranges whose
// boundaries are moved forward to the next newline, each thread parses its range with
// std::from_chars into a private buffer (rows counted first so the output is written
// in place), and the result is one contiguous row-major double array owned by the
// caller (sysml_free).
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <string>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace {

struct Mapped {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  bool open(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    n = (size_t)st.st_size;
    if (n == 0) return true;
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) return false;
    madvise(m, n, MADV_SEQUENTIAL);
    p = (const char*)m;
    return true;
  }
  ~Mapped() {
    if (p) munmap((void*)p, n);
    if (fd >= 0) ::close(fd);
  }
};

inline const char* skip_ws(const char* s, const char* e) {
  while (s < e && (*s == ' ' || *s == '\t' || *s == '\r')) ++s;
  return s;
}

// parse one double in [s, e); empty field -> 0 (the CSV reader's default fill value)
inline const char* parse_double(const char* s, const char* e, double& v, char sep = ',') {
  s = skip_ws(s, e);
  if (s >= e || *s == '\n' || *s == sep) {
    v = 0.0;
    return s;
  }
  if (*s == '+') ++s;
  auto r = std::from_chars(s, e, v);
  if (r.ec != std::errc()) {
    // Java-style literals: Infinity / -Infinity / NaN, quoted numbers
    if (*s == '"') return parse_double(s + 1, e, v, sep);
    bool neg = (*s == '-');
    const char* t = s + (neg ? 1 : 0);
    if (e - t >= 8 && std::strncmp(t, "Infinity", 8) == 0) {
      v = neg ? -INFINITY : INFINITY;
      return t + 8;
    }
    if (e - t >= 3 && (std::strncmp(t, "NaN", 3) == 0 || std::strncmp(t, "nan", 3) == 0)) {
      v = NAN;
      return t + 3;
    }
    v = NAN;
    while (s < e && *s != sep && *s != '\n') ++s;
    return s;
  }
  s = r.ptr;
  if (s < e && *s == '"') ++s;
  return s;
}

std::vector<size_t> split_lines(const char* p, size_t n, size_t begin, int parts) {
  std::vector<size_t> b(parts + 1, n);
  b[0] = begin;
  for (int i = 1; i < parts; ++i) {
    size_t x = begin + (n - begin) * i / parts;
    if (x < b[i - 1]) x = b[i - 1];
    while (x < n && p[x - 1] != '\n') ++x;
    b[i] = x;
  }
  b[parts] = n;
  return b;
}

size_t count_rows(const char* p, size_t a, size_t z) {
  size_t rows = 0;
  size_t i = a;
  while (i < z) {
    const char* nl = (const char*)memchr(p + i, '\n', z - i);
    size_t end = nl ? (size_t)(nl - p) : z;
    // skip blank lines
    bool blank = true;
    for (size_t k = i; k < end; ++k)
      if (p[k] != ' ' && p[k] != '\t' && p[k] != '\r') { blank = false; break; }
    if (!blank) ++rows;
    i = end + 1;
  }
  return rows;
}

}  // namespace

extern "C" {

void sysml_free(void* p) { std::free(p); }

// CSV of doubles -> row-major buffer of data rows [row_lo, row_hi) (all rows: 0, INT64_MAX).
// Every thread counts the rows of its byte range (memchr only), then only the ranges that
// overlap the requested rows are parsed -- a rank of an SPMD run parses just its own row
// block.  *total_out receives the file's row count.  Returns rows*cols or -1 on error.
int64_t sysml_parse_csv_rows(const char* path, char sep, int header, int64_t row_lo, int64_t row_hi,
                             int64_t* rows_out, int64_t* cols_out, int64_t* total_out, double** out,
                             int threads) {
  Mapped f;
  if (!f.open(path)) return -1;
  const char* p = f.p;
  size_t n = f.n;
  size_t start = 0;
  if (header && n) {
    const char* nl = (const char*)memchr(p, '\n', n);
    start = nl ? (size_t)(nl - p) + 1 : n;
  }
  // columns from the first data line
  int64_t cols = 0;
  {
    size_t i = start;
    while (i < n && (p[i] == '\n' || p[i] == '\r')) ++i;
    size_t e = i;
    while (e < n && p[e] != '\n') ++e;
    if (e > i) {
      cols = 1;
      for (size_t k = i; k < e; ++k)
        if (p[k] == sep) ++cols;
    }
  }
  if (threads < 1) threads = 1;
  if (n - start < (size_t)1 << 20) threads = 1;
  auto b = split_lines(p, n, start, threads);
  std::vector<size_t> rcount(threads);
  {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back([&, t] { rcount[t] = count_rows(p, b[t], b[t + 1]); });
    for (auto& t : ts) t.join();
  }
  std::vector<size_t> roff(threads + 1, 0);
  for (int t = 0; t < threads; ++t) roff[t + 1] = roff[t] + rcount[t];
  int64_t total = (int64_t)roff[threads];
  if (row_lo < 0) row_lo = 0;
  if (row_hi > total) row_hi = total;
  if (row_lo > row_hi) row_lo = row_hi;
  int64_t rows = row_hi - row_lo;
  double* buf = (double*)std::malloc(sizeof(double) * (size_t)std::max<int64_t>(rows * cols, 1));
  if (!buf) return -1;
  bool bad = false;
  {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
      ts.emplace_back([&, t] {
        int64_t r = (int64_t)roff[t];
        if (r >= row_hi || (int64_t)roff[t + 1] <= row_lo) return;
        size_t i = b[t], z = b[t + 1];
        while (i < z && r < row_hi) {
          const char* nl = (const char*)memchr(p + i, '\n', z - i);
          size_t end = nl ? (size_t)(nl - p) : z;
          const char* s = p + i;
          const char* e = p + end;
          const char* q = skip_ws(s, e);
          if (q < e) {
            const int64_t row = r++;            // data row index in the file
            if (row < row_lo) {
              i = end + 1;
              continue;
            }
            double* o = buf + (row - row_lo) * cols;
            int64_t c = 0;
            while (c < cols) {
              double v;
              s = parse_double(s, e, v, sep);
              o[c++] = v;
              s = skip_ws(s, e);
              if (s < e && *s == sep) ++s;
              else break;
            }
            for (; c < cols; ++c) o[c] = 0.0;   // short line: fill
          }
          i = end + 1;
        }
        (void)bad;
      });
    for (auto& t : ts) t.join();
  }
  *rows_out = rows;
  *cols_out = cols;
  *total_out = total;
  *out = buf;
  return rows * cols;
}

int64_t sysml_parse_csv(const char* path, char sep, int header, int64_t* rows_out, int64_t* cols_out,
                        double** out, int threads) {
  int64_t total;
  return sysml_parse_csv_rows(path, sep, header, 0, INT64_MAX, rows_out, cols_out, &total, out, threads);
}

// "i j v" text cell format -> n x 3 row-major buffer; returns n or -1.
int64_t sysml_parse_ijv(const char* path, double** out, int threads) {
  Mapped f;
  if (!f.open(path)) return -1;
  const char* p = f.p;
  size_t n = f.n;
  if (threads < 1) threads = 1;
  if (n < (size_t)1 << 20) threads = 1;
  auto b = split_lines(p, n, 0, threads);
  std::vector<size_t> rcount(threads);
  {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back([&, t] { rcount[t] = count_rows(p, b[t], b[t + 1]); });
    for (auto& t : ts) t.join();
  }
  std::vector<size_t> roff(threads + 1, 0);
  for (int t = 0; t < threads; ++t) roff[t + 1] = roff[t] + rcount[t];
  size_t rows = roff[threads];
  double* buf = (double*)std::malloc(sizeof(double) * std::max<size_t>(rows * 3, 1));
  if (!buf) return -1;
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t] {
      size_t i = b[t], z = b[t + 1];
      double* o = buf + roff[t] * 3;
      while (i < z) {
        const char* nl = (const char*)memchr(p + i, '\n', z - i);
        size_t end = nl ? (size_t)(nl - p) : z;
        const char* s = p + i;
        const char* e = p + end;
        if (skip_ws(s, e) < e) {
          for (int c = 0; c < 3; ++c) {
            double v;
            s = parse_double(s, e, v, ' ');
            o[c] = v;
          }
          o += 3;
        }
        i = end + 1;
      }
    });
  for (auto& t : ts) t.join();
  *out = buf;
  return (int64_t)rows;
}

// ---------------------------------------------------------------------------------------
// Writers (reference: runtime/io/WriterTextCSVParallel.java, WriterTextCellParallel.java):
// cells formatted like java.lang.Double.toString from the shortest round-trip digits
// (std::to_chars), rows formatted in parallel into per-thread buffers, written in order.
// ---------------------------------------------------------------------------------------
static int java_double(double d, char* out) {
  if (std::isnan(d)) { std::memcpy(out, "NaN", 3); return 3; }
  if (std::isinf(d)) {
    if (d > 0) { std::memcpy(out, "Infinity", 8); return 8; }
    std::memcpy(out, "-Infinity", 9); return 9;
  }
  if (d == 0.0) {
    if (std::signbit(d)) { std::memcpy(out, "-0.0", 4); return 4; }
    std::memcpy(out, "0.0", 3); return 3;
  }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), d, std::chars_format::scientific);
  char* e = std::find(buf, r.ptr, 'e');
  int exp10 = 0;
  std::from_chars(e + 1 + (e[1] == '+'), r.ptr, exp10);     // [e+1, r.ptr): not NUL-terminated
  char digits[32];
  int nd = 0;
  int k = 0;
  bool neg = false;
  if (buf[0] == '-') { neg = true; k = 1; }
  for (; buf + k < e; ++k)
    if (buf[k] != '.') digits[nd++] = buf[k];
  while (nd > 1 && digits[nd - 1] == '0') --nd;
  int o = 0;
  if (neg) out[o++] = '-';
  const double a = std::fabs(d);
  if (a >= 1e-3 && a < 1e7) {
    if (exp10 >= 0) {                      // ddd.ddd
      for (int i = 0; i <= exp10; ++i) out[o++] = i < nd ? digits[i] : '0';
      out[o++] = '.';
      if (nd > exp10 + 1) for (int i = exp10 + 1; i < nd; ++i) out[o++] = digits[i];
      else out[o++] = '0';
    } else {                               // 0.000ddd
      out[o++] = '0'; out[o++] = '.';
      for (int i = 0; i < -exp10 - 1; ++i) out[o++] = '0';
      for (int i = 0; i < nd; ++i) out[o++] = digits[i];
    }
    return o;
  }
  out[o++] = digits[0];
  out[o++] = '.';
  if (nd > 1) for (int i = 1; i < nd; ++i) out[o++] = digits[i];
  else out[o++] = '0';
  out[o++] = 'E';
  auto r2 = std::to_chars(out + o, out + o + 8, exp10);
  return (int)(r2.ptr - out);
}

// mode 0: dense rows joined by `sep` (csv); mode 1: "i j v" lines of the non-zeros (text / mm)
int64_t sysml_write_cells(const char* path, const double* a, int64_t rows, int64_t cols, int mode, char sep,
                          int append, int threads) {
  FILE* f = std::fopen(path, append ? "ab" : "wb");
  if (!f) return -1;
  if (threads < 1) threads = 1;
  const int64_t chunk = 4096;
  std::vector<std::string> bufs(threads);
  for (int64_t base = 0; base < rows; base += chunk * threads) {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) {
      th.emplace_back([&, t]() {
        std::string& b = bufs[t];
        b.clear();
        char cell[64], num[32];
        const int64_t r0 = base + t * chunk, r1 = std::min(rows, r0 + chunk);
        for (int64_t i = r0; i < r1; ++i) {
          const double* row = a + i * cols;
          if (mode == 0) {
            for (int64_t j = 0; j < cols; ++j) {
              if (j) b.push_back(sep);
              const int n = java_double(row[j], cell);
              b.append(cell, (size_t)n);
            }
            b.push_back('\n');
          } else {
            for (int64_t j = 0; j < cols; ++j) {
              if (row[j] == 0.0) continue;
              auto p = std::to_chars(num, num + 32, i + 1);
              b.append(num, p.ptr - num);
              b.push_back(' ');
              p = std::to_chars(num, num + 32, j + 1);
              b.append(num, p.ptr - num);
              b.push_back(' ');
              const int n = java_double(row[j], cell);
              b.append(cell, (size_t)n);
              b.push_back('\n');
            }
          }
        }
      });
    }
    for (auto& x : th) x.join();
    for (int t = 0; t < threads; ++t)
      if (!bufs[t].empty() && std::fwrite(bufs[t].data(), 1, bufs[t].size(), f) != bufs[t].size()) {
        std::fclose(f);
        return -2;
      }
  }
  return std::fclose(f) == 0 ? 0 : -3;
}

// one Java-formatted double (tests / scalar writes)
int sysml_java_double(double d, char* out) { return java_double(d, out); }

}  // extern "C"
