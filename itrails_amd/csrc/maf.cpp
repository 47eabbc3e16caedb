// maf.cpp — streaming MAF reader for the decoding core.
//
// Replaces maf_parser / parse_coordinates (read_data.py:94-220), which walk Biopython's
// AlignIO MAF records in Python and map every column with a 625-entry list search.  Here
// the file is memory-mapped and scanned once; every column becomes its uint16 symbol by a
// 5^4 table lookup, written straight into the concatenated observation array the sweeps
// consume (blocks back to back + offsets).
//
// Semantics kept from the reference (with Biopython's MafIO record model):
//  * a block = lines from an 'a' line to the next blank line / 'a' line; only 's' lines
//    carry sequences (src start size strand srcSize text); '#', 'i', 'e', 'q' lines are
//    skipped;
//  * species of a record = src up to the first '.'; a block is kept iff all 4 species of
//    sp_lst have a record (a repeated species: the last record wins), read_data.py:106-110;
//  * column string = the 4 species' characters in sp_lst order, '-' -> 'N', upper-cased;
//    anything outside A/C/T/G/N raises (list.index ValueError, read_data.py:113-115);
//  * block length = length of the block's last record (read_data.py:111); records of one
//    block must have equal lengths (Biopython refuses ragged alignments);
//  * coordinates (parse_coordinates, read_data.py:150-220): kept iff exactly 4 records
//    belong to sp_lst; position of every non-gap reference character, counting up from
//    `start` on '+', down from srcSize - start on '-', -9 for gaps and for blocks without
//    the reference.
#include <ctype.h>
#include <fcntl.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "maf.h"

namespace itr {

namespace {

// letter -> code A=0 C=1 T=2 G=3 N=4 ('-' is N), 0xFF: not in the alphabet
struct Codes {
  uint8_t code[256];
  uint16_t sym[625];  // (c0*125 + c1*25 + c2*5 + c3) -> symbol index (read_data.py:6-24)
  Codes() {
    memset(code, 0xFF, sizeof code);
    const char* up = "ACTGN";
    const char* lo = "actgn";
    for (int i = 0; i < 5; ++i) {
      code[(uint8_t)up[i]] = (uint8_t)i;
      code[(uint8_t)lo[i]] = (uint8_t)i;
    }
    code[(uint8_t)'-'] = 4;
    int next_n = 256;  // N-containing strings in 5-letter enumeration order
    for (int a = 0; a < 5; ++a)
      for (int b = 0; b < 5; ++b)
        for (int c = 0; c < 5; ++c)
          for (int d = 0; d < 5; ++d) {
            const int k = ((a * 5 + b) * 5 + c) * 5 + d;
            if (a < 4 && b < 4 && c < 4 && d < 4)
              sym[k] = (uint16_t)(((a * 4 + b) * 4 + c) * 4 + d);
            else
              sym[k] = (uint16_t)next_n++;
          }
  }
};
const Codes kCodes;

struct Rec {
  const char* src;
  size_t src_len;
  long long start, src_size;
  int strand;
  const char* text;
  size_t len;
};

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r'; }

// split an 's' line into its 7 fields
bool parse_s(const char* p, const char* end, Rec* r) {
  const char* f[7];
  size_t fl[7];
  int nf = 0;
  while (p < end && nf < 7) {
    while (p < end && is_space(*p)) ++p;
    if (p >= end) break;
    const char* s = p;
    while (p < end && !is_space(*p)) ++p;
    f[nf] = s;
    fl[nf] = (size_t)(p - s);
    ++nf;
  }
  if (nf < 7) return false;
  r->src = f[1];
  r->src_len = fl[1];
  r->start = strtoll(std::string(f[2], fl[2]).c_str(), nullptr, 10);
  r->strand = (fl[4] == 1 && f[4][0] == '-') ? -1 : 1;
  r->src_size = strtoll(std::string(f[5], fl[5]).c_str(), nullptr, 10);
  r->text = f[6];
  r->len = fl[6];
  return true;
}

}  // namespace

// Scan [data, end) — whole blocks only — appending to *out.
static int scan(const char* data, const char* end, const char* const species[4],
                const char* ref, MafResult* out, std::string* err) {
  out->obs.clear();
  out->off.assign(1, 0);
  out->coords.clear();
  out->coord_off.assign(1, 0);
  size_t sp_len[4];
  for (int k = 0; k < 4; ++k) sp_len[k] = strlen(species[k]);
  const size_t ref_len = ref ? strlen(ref) : 0;

  std::vector<Rec> recs;
  int rc = 0;
  auto species_of = [&](const Rec& r, const char* name, size_t nlen) {
    size_t dot = 0;
    while (dot < r.src_len && r.src[dot] != '.') ++dot;
    return dot == nlen && memcmp(r.src, name, nlen) == 0;
  };
  auto flush = [&]() -> int {
    if (recs.empty()) return 0;
    // ---- observations (maf_parser)
    const Rec* pick[4] = {nullptr, nullptr, nullptr, nullptr};
    int in_list = 0;
    for (const Rec& r : recs) {
      bool member = false;
      for (int k = 0; k < 4; ++k)
        if (species_of(r, species[k], sp_len[k])) {
          pick[k] = &r;  // the last record of a species wins
          member = true;
        }
      in_list += member;
    }
    const size_t len = recs.back().len;
    for (const Rec& r : recs)
      if (r.len != len) {
        *err = "alignment block with records of different lengths";
        return 1;
      }
    if (pick[0] && pick[1] && pick[2] && pick[3]) {
      const size_t base = out->obs.size();
      out->obs.resize(base + len);
      uint16_t* o = out->obs.data() + base;
      const uint8_t* s0 = (const uint8_t*)pick[0]->text;
      const uint8_t* s1 = (const uint8_t*)pick[1]->text;
      const uint8_t* s2 = (const uint8_t*)pick[2]->text;
      const uint8_t* s3 = (const uint8_t*)pick[3]->text;
      for (size_t i = 0; i < len; ++i) {
        const uint8_t a = kCodes.code[s0[i]], b = kCodes.code[s1[i]], c = kCodes.code[s2[i]],
                      d = kCodes.code[s3[i]];
        if ((a | b | c | d) == 0xFF || a > 4 || b > 4 || c > 4 || d > 4) {
          std::string col;
          for (const uint8_t* s : {s0, s1, s2, s3}) col += (char)toupper(s[i] == '-' ? 'N' : s[i]);
          *err = "'" + col + "' is not in list";
          return 2;
        }
        o[i] = kCodes.sym[((a * 5 + b) * 5 + c) * 5 + d];
      }
      out->off.push_back((int64_t)out->obs.size());
    }
    // ---- coordinates (parse_coordinates)
    if (ref && in_list == 4) {
      const Rec* rr = nullptr;
      const Rec* last_member = nullptr;
      for (const Rec& r : recs) {
        for (int k = 0; k < 4; ++k)
          if (species_of(r, species[k], sp_len[k])) last_member = &r;
        if (species_of(r, ref, ref_len)) rr = &r;
      }
      const size_t base = out->coords.size();
      if (rr) {
        out->coords.resize(base + rr->len);
        long long pos = rr->strand == 1 ? rr->start : rr->src_size - rr->start;
        for (size_t i = 0; i < rr->len; ++i) {
          if (rr->text[i] != '-') {
            out->coords[base + i] = pos;
            pos += rr->strand;
          } else {
            out->coords[base + i] = -9;
          }
        }
      } else {
        out->coords.resize(base + last_member->len, -9);
      }
      out->coord_off.push_back((int64_t)out->coords.size());
    }
    recs.clear();
    return 0;
  };

  const char* p = data;
  while (p < end) {
    const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
    const char* le = nl ? nl : end;
    const char* q = p;
    while (q < le && is_space(*q)) ++q;
    if (q == le) {  // blank line ends a block
      if ((rc = flush())) break;
    } else if (*q == 'a' && (q + 1 == le || is_space(q[1]))) {
      if ((rc = flush())) break;
    } else if (*q == 's' && q + 1 < le && is_space(q[1])) {
      Rec r;
      if (!parse_s(q, le, &r)) {
        *err = "malformed 's' line";
        rc = 1;
        break;
      }
      recs.push_back(r);
    }
    p = nl ? nl + 1 : end;
  }
  if (!rc) rc = flush();
  return rc;
}


// start of the first block line ('a' at the start of a line) at or after p, or end
static const char* next_block(const char* p, const char* begin, const char* end) {
  while (p < end) {
    if ((p == begin || p[-1] == '\n') && *p == 'a' && (p + 1 == end || is_space(p[1]) || p[1] == '\n'))
      return p;
    const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
    if (!nl) return end;
    p = nl + 1;
  }
  return end;
}

int maf_read(const char* path, const char* const species[4], const char* ref, MafResult* out,
             std::string* err) {
  out->obs.clear();
  out->off.assign(1, 0);
  out->coords.clear();
  out->coord_off.assign(1, 0);
  int fd = open(path, O_RDONLY);
  if (fd < 0) {
    *err = std::string("cannot open ") + path;
    return 1;
  }
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    *err = "stat failed";
    return 1;
  }
  const size_t size = (size_t)st.st_size;
  if (size == 0) {
    close(fd);
    return 0;
  }
  void* map = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (map == MAP_FAILED) {
    *err = "mmap failed";
    return 1;
  }
  madvise(map, size, MADV_SEQUENTIAL);
  const char* data = (const char*)map;
  const char* end = data + size;

  // split at block starts into up to 16 ranges scanned in parallel, merged in file order
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (size < ((size_t)8 << 20)) nt = 1;
  if (const char* e = getenv("ITR_MAF_THREADS")) nt = std::max(1, std::min(64, atoi(e)));
  std::vector<const char*> cut{data};
  for (unsigned t = 1; t < nt; ++t) {
    const char* c = next_block(std::max(cut.back(), data + size / nt * t), data, end);
    if (c > cut.back() && c < end) cut.push_back(c);
  }
  cut.push_back(end);
  const size_t nr = cut.size() - 1;
  std::vector<MafResult> part(nr);
  std::vector<std::string> perr(nr);
  std::vector<int> prc(nr, 0);
  std::vector<std::thread> th;
  for (size_t r = 0; r < nr; ++r)
    th.emplace_back([&, r] { prc[r] = scan(cut[r], cut[r + 1], species, ref, &part[r], &perr[r]); });
  for (auto& t : th) t.join();
  munmap(map, size);
  for (size_t r = 0; r < nr; ++r)
    if (prc[r]) {  // the first failure in file order, as a sequential reader would report
      *err = perr[r];
      out->off.assign(1, 0);
      return prc[r];
    }
  size_t nobs = 0, ncrd = 0;
  for (auto& p : part) {
    nobs += p.obs.size();
    ncrd += p.coords.size();
  }
  out->obs.reserve(nobs);
  out->coords.reserve(ncrd);
  for (auto& p : part) {
    const int64_t b = (int64_t)out->obs.size(), bc = (int64_t)out->coords.size();
    out->obs.insert(out->obs.end(), p.obs.begin(), p.obs.end());
    for (size_t k = 1; k < p.off.size(); ++k) out->off.push_back(b + p.off[k]);
    out->coords.insert(out->coords.end(), p.coords.begin(), p.coords.end());
    for (size_t k = 1; k < p.coord_off.size(); ++k) out->coord_off.push_back(bc + p.coord_off[k]);
  }
  return 0;
}

}  // namespace itr
