// TEST-ONLY differential check of the planner's strict base64 decoder (AVX2
// blocks + scalar tail, host/gojson.cpp b64_decode_strict_append) against the
// Go-semantics decoder (b64_decode_append, newline skipping excluded) on random
// valid, corrupted and alphabet-substituted encodings.  Exit 0 = no mismatch.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>
#include "../../fabric-token-sdk_amd/csrc/host/gojson.h"
using namespace ftsh;
int main() {
  std::mt19937 rng(1);
  const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  long bad = 0, cases = 0;
  for (int it = 0; it < 200000; it++) {
    size_t len = rng() % 300;
    std::vector<uint8_t> raw(len);
    for (auto& b : raw) b = rng();
    std::string enc; b64_encode(raw.data(), raw.size(), enc);
    int mode = rng() % 3;
    if (mode == 1 && !enc.empty()) enc[rng() % enc.size()] = (char)(rng() % 256);  // any byte anywhere
    if (mode == 2 && !enc.empty()) enc[rng() % enc.size()] = A[rng() % 64];
    std::vector<uint8_t> o1 = {7, 7}, o2 = {7, 7};
    bool r1 = b64_decode_strict_append(enc.data(), enc.size(), o1);
    // reference: the scalar strict rule = Go semantics without newline skipping
    bool hasnl = enc.find('\r') != std::string::npos || enc.find('\n') != std::string::npos;
    bool r2 = !hasnl && b64_decode_append(enc.data(), enc.size(), o2);
    cases++;
    if (r1 != r2 || (r1 && o1 != o2)) { bad++; if (bad < 5) printf("mismatch len %zu mode %d r1 %d r2 %d\n", enc.size(), mode, r1, r2); }
  }
  printf("cases %ld mismatches %ld\n", cases, bad);
  return bad != 0;
}
