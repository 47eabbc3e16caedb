// writers.cpp — result files of the decoding CLIs.
//
// Byte-compatible with the reference's csv.writer output (excel dialect: ',' separated,
// "\r\n" line ends, values through str()):
//  * Viterbi segments  (workflow_viterbi.py:690-743): Block_idx,position_start,position_end,
//    most_likely_state — one row per run of equal states; states print as floats ("5.0",
//    the reference's float64 paths); with reference coordinates the run bounds are genomic
//    positions and gap columns (-9) extend / split runs exactly as the reference's loop does.
//  * posterior table   (workflow_posterior.py:697-716): alignment_block_idx,position_idx,
//    prob_state_0..N-1, one row per column, every probability printed like Python's
//    repr(float) (shortest round-trip digits; exponent form below 1e-4 and from 1e16).
//    At 10 Mbp x 133 states this is ~1.3e9 numbers: rows are formatted by up to 16 threads
//    into per-chunk buffers and written in order.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <string>
#include <thread>
#include <vector>

#include "writers.h"

namespace itr {

// Python repr(float) (float_repr_style 'short'): shortest digits that round-trip; fixed
// notation when -4 <= exponent < 16, else d[.ddd]e±XX with at least two exponent digits.
int format_pyfloat(double x, char* out) {
  if (std::isnan(x)) {
    memcpy(out, "nan", 3);
    return 3;
  }
  if (std::isinf(x)) {
    if (x < 0) {
      memcpy(out, "-inf", 4);
      return 4;
    }
    memcpy(out, "inf", 3);
    return 3;
  }
  char* o = out;
  if (std::signbit(x)) {
    *o++ = '-';
    x = -x;
  }
  if (x == 0.0) {
    memcpy(o, "0.0", 3);
    return (int)(o - out) + 3;
  }
  char buf[40];
  auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
  // buf = d[.ddd]e±XX
  char digits[24];
  int nd = 0;
  const char* p = buf;
  while (*p != 'e' && p < r.ptr) {
    if (*p != '.') digits[nd++] = *p;
    ++p;
  }
  int exp10 = 0;
  {
    ++p;  // 'e'
    const bool neg = *p == '-';
    ++p;
    while (p < r.ptr) exp10 = exp10 * 10 + (*p++ - '0');
    if (neg) exp10 = -exp10;
  }
  const int decpt = exp10 + 1;  // digits before the decimal point
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      *o++ = '0';
      *o++ = '.';
      for (int i = 0; i < -decpt; ++i) *o++ = '0';
      memcpy(o, digits, nd);
      o += nd;
    } else if (decpt >= nd) {
      memcpy(o, digits, nd);
      o += nd;
      for (int i = nd; i < decpt; ++i) *o++ = '0';
      *o++ = '.';
      *o++ = '0';
    } else {
      memcpy(o, digits, decpt);
      o += decpt;
      *o++ = '.';
      memcpy(o, digits + decpt, nd - decpt);
      o += nd - decpt;
    }
  } else {
    *o++ = digits[0];
    if (nd > 1) {
      *o++ = '.';
      memcpy(o, digits + 1, nd - 1);
      o += nd - 1;
    }
    *o++ = 'e';
    int e = decpt - 1;
    *o++ = e < 0 ? '-' : '+';
    if (e < 0) e = -e;
    char eb[8];
    int ne = 0;
    do {
      eb[ne++] = (char)('0' + e % 10);
      e /= 10;
    } while (e);
    if (ne < 2) eb[ne++] = '0';
    while (ne) *o++ = eb[--ne];
  }
  return (int)(o - out);
}

namespace {

inline void put_i64(std::string& s, long long v) {
  char b[24];
  auto r = std::to_chars(b, b + sizeof b, v);
  s.append(b, r.ptr);
}
inline void put_state(std::string& s, int v) {  // float64 state index, str() form
  put_i64(s, v);
  s.append(".0");
}

struct File {
  FILE* f = nullptr;
  ~File() {
    if (f) fclose(f);
  }
};

}  // namespace

int write_viterbi_csv(const char* path, const uint8_t* states, const int64_t* off,
                      int64_t nblocks, const int64_t* coords, std::string* err) {
  File fh;
  fh.f = fopen(path, "wb");
  if (!fh.f) {
    *err = std::string("cannot open ") + path + " for writing";
    return 1;
  }
  std::string s = "Block_idx,position_start,position_end,most_likely_state\r\n";
  auto row = [&](int64_t blk, long long a, long long b, int st) {
    put_i64(s, blk);
    s.push_back(',');
    put_i64(s, a);
    s.push_back(',');
    put_i64(s, b);
    s.push_back(',');
    put_state(s, st);
    s.append("\r\n");
    if (s.size() > ((size_t)1 << 22)) {
      fwrite(s.data(), 1, s.size(), fh.f);
      s.clear();
    }
  };
  for (int64_t k = 0; k < nblocks; ++k) {
    const int64_t c0 = off[k], T = off[k + 1] - off[k];
    if (T == 0) continue;
    const uint8_t* res = states + c0;
    if (!coords) {
      long long seg = 0;
      int cur = res[0];
      for (int64_t pos = 1; pos < T; ++pos)
        if (res[pos] != cur) {
          row(k, seg, pos - 1, cur);
          seg = pos;
          cur = res[pos];
        }
      row(k, seg, T - 1, cur);
    } else {
      const int64_t* rc = coords + c0;
      int64_t first = -1;
      for (int64_t i = 0; i < T; ++i)
        if (rc[i] != -9) {
          first = i;
          break;
        }
      if (first < 0) continue;
      long long seg = rc[first], cur_nn = seg;
      int cur = res[first];
      for (int64_t pos = first; pos < T; ++pos) {
        if (seg == -9) {
          seg = rc[pos];
          cur = res[pos];
          cur_nn = seg;
          continue;
        }
        if (res[pos] != cur) {
          row(k, seg, cur_nn, cur);
          seg = rc[pos];
          cur = res[pos];
        }
        cur_nn = rc[pos] != -9 ? rc[pos] : cur_nn;
      }
      if (!(seg == cur_nn && cur_nn == -9)) row(k, seg, cur_nn, cur);
    }
  }
  fwrite(s.data(), 1, s.size(), fh.f);
  if (ferror(fh.f)) {
    *err = "write failed";
    return 1;
  }
  return 0;
}

int write_posterior_csv(const char* path, const double* post, int n_states, const int64_t* off,
                        int64_t nblocks, const int64_t* coords, int threads, std::string* err) {
  File fh;
  fh.f = fopen(path, "wb");
  if (!fh.f) {
    *err = std::string("cannot open ") + path + " for writing";
    return 1;
  }
  std::string head = "alignment_block_idx,position_idx";
  for (int i = 0; i < n_states; ++i) head += ",prob_state_" + std::to_string(i);
  head += "\r\n";
  fwrite(head.data(), 1, head.size(), fh.f);
  const int64_t total = nblocks > 0 ? off[nblocks] : 0;
  // block of every column (rows carry their block index)
  const int nt = std::max(1, std::min(threads > 0 ? threads : 16,
                                      (int)std::thread::hardware_concurrency()));
  const int64_t chunk = 1 << 14;  // rows per formatting task
  // two rounds of per-thread buffers: the workers format round k + 1 while this thread
  // writes round k, so the (serial) file writes overlap the (parallel) formatting.  The
  // rounds alternate by index; each worker gets its destination string by value before it
  // starts, so nothing it touches is rebound while it runs.
  std::vector<std::string> bufs[2] = {std::vector<std::string>(nt), std::vector<std::string>(nt)};
  auto launch = [&](int64_t r0, int round) {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) {
      std::string* dst = &bufs[round][t];
      th.emplace_back([&, r0, t, dst] {
        std::string& s = *dst;
        s.clear();
        const int64_t a = r0 + t * chunk, b = std::min(total, a + chunk);
        if (a >= b) return;
        s.reserve((size_t)(b - a) * (n_states * 22 + 16));
        int64_t blk = std::upper_bound(off, off + nblocks + 1, a) - off - 1;
        char num[40];
        for (int64_t c = a; c < b; ++c) {
          while (off[blk + 1] <= c) ++blk;
          put_i64(s, blk);
          s.push_back(',');
          put_i64(s, coords ? coords[c] : c - off[blk]);
          const double* rowp = post + c * n_states;
          for (int i = 0; i < n_states; ++i) {
            s.push_back(',');
            s.append(num, format_pyfloat(rowp[i], num));
          }
          s.append("\r\n");
        }
      });
    }
    return th;
  };
  const int64_t step = chunk * nt;
  std::vector<std::thread> th = launch(0, 0);
  int round = 0;
  for (int64_t r0 = 0; r0 < total; r0 += step, round ^= 1) {
    for (auto& x : th) x.join();
    th = r0 + step < total ? launch(r0 + step, round ^ 1) : std::vector<std::thread>();
    for (int t = 0; t < nt; ++t) fwrite(bufs[round][t].data(), 1, bufs[round][t].size(), fh.f);
  }
  for (auto& x : th) x.join();
  if (ferror(fh.f)) {
    *err = "write failed";
    return 1;
  }
  return 0;
}

}  // namespace itr
