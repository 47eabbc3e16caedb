// maf.h — streaming MAF reader (maf.cpp).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace itr {

struct MafResult {
  std::vector<uint16_t> obs;       // symbols of the kept blocks, back to back
  std::vector<int64_t> off;        // [kept blocks + 1]
  std::vector<int64_t> coords;     // reference coordinates (if requested)
  std::vector<int64_t> coord_off;  // [coordinate blocks + 1]
};

// 0 ok; 1 I/O or format error; 2 a column outside the alphabet (the reference's ValueError)
int maf_read(const char* path, const char* const species[4], const char* ref, MafResult* out,
             std::string* err);

}  // namespace itr
