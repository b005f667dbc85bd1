// Go encoding/json restated for the zkatdlog proof wire format (host side of
// the product boundary).  Semantics reproduced:
//   * struct fields match object keys exactly or case-insensitively; a later
//     duplicate key overwrites an earlier one; unknown keys are ignored;
//   * JSON null leaves pointers / slices nil;
//   * []byte is standard base64 with padding, '\r' and '\n' skipped;
//   * mathlib elements are {"curve": <int>, "element": <[]byte>}.
// The parser builds a flat DOM (node indices into one vector) per document.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

namespace ftsh {

enum JType : uint8_t { J_NULL, J_BOOL, J_NUM, J_STR, J_ARR, J_OBJ };

struct JNode {
  JType type;
  uint8_t bval;
  uint32_t first;   // ARR/OBJ: index of first child in kids[]; STR/NUM: offset into text pool
  uint32_t count;   // ARR/OBJ: number of children; STR/NUM: length
};

struct JDoc {
  std::vector<JNode> nodes;
  std::vector<uint32_t> kids;      // OBJ: pairs (key node, value node); ARR: value nodes
  std::string pool;                // unescaped strings and number tokens
  bool parse(const uint8_t* p, size_t n);  // false on syntax error

  uint32_t root() const { return (uint32_t)nodes.size() - 1; }
  const JNode& at(uint32_t i) const { return nodes[i]; }
  // Go struct-field lookup on an object node: returns node index or -1
  int64_t field(uint32_t obj, const char* name) const;
  const char* str(uint32_t i) const { return pool.data() + nodes[i].first; }
  uint32_t len(uint32_t i) const { return nodes[i].count; }
  uint32_t elem(uint32_t arr, uint32_t k) const { return kids[nodes[arr].first + k]; }
};

// base64.StdEncoding.DecodeString ('\r','\n' skipped); false if illegal
bool b64_decode(const char* s, size_t n, std::vector<uint8_t>& out);
void b64_encode(const uint8_t* p, size_t n, std::string& out);

// Result of decoding a JSON value into a Go field of the given kind.
enum DecStatus : uint8_t { D_OK = 0, D_NIL = 1, D_ERR = 2, D_PANIC = 3 };

struct ElemBytes {
  DecStatus st;
  std::vector<uint8_t> raw;  // element bytes (D_OK)
};

// mathlib element (Zr/G1/G2) UnmarshalJSON: curve must be BN254 (= 1); any
// other id makes the reference panic on first use (driver type assertion).
ElemBytes dec_elem(const JDoc& d, int64_t node);
// []byte field
DecStatus dec_bytes(const JDoc& d, int64_t node, std::vector<uint8_t>& out);
// int field (Go: number without fraction/exponent)
DecStatus dec_int(const JDoc& d, int64_t node, int64_t& out);
// string field
DecStatus dec_string(const JDoc& d, int64_t node, std::string& out);

}  // namespace ftsh
