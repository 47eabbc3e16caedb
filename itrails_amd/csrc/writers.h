// writers.h — CSV result writers (writers.cpp).
#pragma once
#include <stdint.h>

#include <string>

namespace itr {

int format_pyfloat(double x, char* out);  // Python repr(float); returns length (<= 32)
int write_viterbi_csv(const char* path, const uint8_t* states, const int64_t* off,
                      int64_t nblocks, const int64_t* coords, std::string* err);
int write_posterior_csv(const char* path, const double* post, int n_states, const int64_t* off,
                        int64_t nblocks, const int64_t* coords, int threads, std::string* err);

}  // namespace itr
