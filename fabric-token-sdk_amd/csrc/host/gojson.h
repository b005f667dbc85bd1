// Go encoding/json restated for the zkatdlog proof wire format (host side of
// the product boundary).  Semantics reproduced (Go 1.18, go.mod:3; SURVEY
// Appendix C.2):
//   * struct fields match object keys exactly, else by Go's foldFunc for the
//     field name (encoding/json/fold.go: ASCII case folding, plus U+017F 'ſ'
//     for s/S and U+212A Kelvin sign for k/K when the name holds those letters);
//     a later duplicate key overwrites an earlier leaf value and merges into an
//     earlier struct / slice-of-struct value (go_merge); unknown keys are ignored;
//   * strings are unquoted as encoding/json unquoteBytes does: escapes decoded,
//     unpaired surrogates and invalid UTF-8 bytes become U+FFFD (one per byte);
//   * JSON null leaves pointers / slices nil;
//   * []byte is standard base64 with padding, '\r' and '\n' skipped;
//   * mathlib elements are {"curve": <int>, "element": <[]byte>}.
// The parser is iterative (nesting up to Go's maxNestingDepth = 10000) and
// builds a flat DOM (node indices into one vector) per document; a JDoc keeps
// its buffers between documents, so a planner thread parses without
// allocating once warm.
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

namespace ftsh {

enum JType : uint8_t { J_NULL, J_BOOL, J_NUM, J_STR, J_ARR, J_OBJ };

struct JNode {
  JType type;
  uint8_t bval;
  uint32_t first;   // ARR/OBJ: index of first child in kids[]; NUM, STR: offset into the text pool
                    // (STR with bval = 1: offset into the parsed source text)
  uint32_t count;   // ARR/OBJ: number of children; STR/NUM: length
};

struct JDoc {
  std::vector<JNode> nodes;
  std::vector<uint32_t> kids;      // OBJ: pairs (key node, value node); ARR: value nodes
  std::string pool;                // unescaped strings and number tokens
  std::vector<uint32_t> tmp;       // parser scratch (children of open containers)
  std::vector<uint64_t> frames;    // parser scratch (open containers)
  bool parse(const uint8_t* p, size_t n);  // false on syntax error

  uint32_t root() const { return (uint32_t)nodes.size() - 1; }
  const JNode& at(uint32_t i) const { return nodes[i]; }
  // Go struct-field lookup on an object node: returns node index or -1
  int64_t field(uint32_t obj, const char* name) const;
  const uint8_t* src = nullptr;    // text of the last parse (plain strings point into it)
  const char* str(uint32_t i) const {
    return nodes[i].type == J_STR && nodes[i].bval ? (const char*)src + nodes[i].first : pool.data() + nodes[i].first;
  }
  uint32_t len(uint32_t i) const { return nodes[i].count; }
  uint32_t elem(uint32_t arr, uint32_t k) const { return kids[nodes[arr].first + k]; }
};

// Duplicate keys of struct-typed fields (Go 1.18 decode.go): a *T field whose
// key occurs again is decoded INTO the struct already there (indirect() keeps a
// non-nil pointer, object() does not zero it), so the occurrences merge key by
// key, a null in between resetting the pointer; a []*T field decodes element i
// into the existing element i and then truncates, and the backing array
// outlives the truncation, so a later, longer array merges into the old
// elements again (an empty array installs a fresh slice, null a nil one).
// go_merge rewrites a parsed document so that each such field (named by a
// schema, recursively) occurs once, holding the merged value -- built from the
// concatenated members of its occurrences, so field()'s last-match lookup then
// gives Go's answer for the leaf fields inside as well.  The document is left
// untouched when nothing needs merging; otherwise the new root is appended
// last (root() stays valid).  A struct field whose value is neither null nor
// an object (an array element neither null nor an object) is left to the
// typed decoder, which reports the type error Unmarshal would return.
enum JFieldKind : uint8_t { JF_STRUCT = 1, JF_SLICE = 2 };
struct JField {
  const char* name;      // nullptr ends a schema
  JFieldKind kind;
  const JField* sub;     // schema of the struct / element struct (may be empty)
};
void go_merge(JDoc& d, const JField* schema);

// Go encoding/json field matching of an (unescaped) object key against an
// ASCII struct field name.
bool go_key_matches(const char* key, size_t klen, const char* name, size_t nlen);

// base64.StdEncoding.DecodeString ('\r','\n' skipped); false if illegal.
// b64_decode_append appends to `out` (which keeps its earlier contents).
bool b64_decode(const char* s, size_t n, std::vector<uint8_t>& out);
bool b64_decode_append(const char* s, size_t n, std::vector<uint8_t>& out);
void b64_encode(const uint8_t* p, size_t n, std::string& out);
// strict form for the canonical fast path: alphabet only, length % 4 == 0,
// padding only at the end (no '\r' / '\n'); false otherwise
bool b64_decode_strict_append(const char* s, size_t n, std::vector<uint8_t>& out);

// Result of decoding a JSON value into a Go field of the given kind.
enum DecStatus : uint8_t { D_OK = 0, D_NIL = 1, D_ERR = 2, D_PANIC = 3 };

struct ElemBytes {
  DecStatus st;
  std::vector<uint8_t> raw;  // element bytes (D_OK)
};

// mathlib element (Zr/G1/G2) UnmarshalJSON: curve must be BN254 (= 1); any
// other id makes the reference panic on first use (driver type assertion).
ElemBytes dec_elem(const JDoc& d, int64_t node);
// Same, decoding the element bytes straight into `dst` at a 16-byte aligned
// offset (returned in off/len; dst is restored on error).
DecStatus dec_elem_into(const JDoc& d, int64_t node, std::vector<uint8_t>& dst, size_t& off, uint32_t& len);
// []byte field
DecStatus dec_bytes(const JDoc& d, int64_t node, std::vector<uint8_t>& out);
// the same appended to `out` (left as it was unless D_OK)
DecStatus dec_bytes_append(const JDoc& d, int64_t node, std::vector<uint8_t>& out);
// dec_elem's status with the element bytes appended to `out` (D_OK / D_PANIC;
// `out` unchanged otherwise) -- no ElemBytes allocation per element
DecStatus dec_elem_append(const JDoc& d, int64_t node, std::vector<uint8_t>& out);
// int field (Go: number without fraction/exponent)
DecStatus dec_int(const JDoc& d, int64_t node, int64_t& out);
// string field
DecStatus dec_string(const JDoc& d, int64_t node, std::string& out);

}  // namespace ftsh
