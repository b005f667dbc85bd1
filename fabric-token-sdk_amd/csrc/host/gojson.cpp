#include "gojson.h"

#include <immintrin.h>

namespace ftsh {

namespace {

constexpr uint32_t MAX_DEPTH = 10000;  // encoding/json scanner.go maxNestingDepth

inline bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }

void put_utf8(std::string& o, uint32_t cp) {
  char b[4];
  if (cp < 0x80) {
    o.push_back((char)cp);
    return;
  }
  if (cp < 0x800) {
    b[0] = (char)(0xC0 | (cp >> 6));
    b[1] = (char)(0x80 | (cp & 0x3F));
    o.append(b, 2);
  } else if (cp < 0x10000) {
    b[0] = (char)(0xE0 | (cp >> 12));
    b[1] = (char)(0x80 | ((cp >> 6) & 0x3F));
    b[2] = (char)(0x80 | (cp & 0x3F));
    o.append(b, 3);
  } else {
    b[0] = (char)(0xF0 | (cp >> 18));
    b[1] = (char)(0x80 | ((cp >> 12) & 0x3F));
    b[2] = (char)(0x80 | ((cp >> 6) & 0x3F));
    b[3] = (char)(0x80 | (cp & 0x3F));
    o.append(b, 4);
  }
}

// unicode/utf8.DecodeRune: returns the rune and its size; invalid -> (U+FFFD, 1)
uint32_t decode_rune(const uint8_t* s, size_t n, size_t& size) {
  size = 1;
  uint8_t b0 = s[0];
  if (b0 < 0x80) return b0;
  auto cont = [&](size_t k, uint8_t lo, uint8_t hi) { return k < n && s[k] >= lo && s[k] <= hi; };
  if (b0 >= 0xC2 && b0 <= 0xDF) {
    if (!cont(1, 0x80, 0xBF)) return 0xFFFD;
    size = 2;
    return ((uint32_t)(b0 & 0x1F) << 6) | (s[1] & 0x3F);
  }
  if (b0 >= 0xE0 && b0 <= 0xEF) {
    uint8_t lo = b0 == 0xE0 ? 0xA0 : 0x80, hi = b0 == 0xED ? 0x9F : 0xBF;
    if (!cont(1, lo, hi) || !cont(2, 0x80, 0xBF)) return 0xFFFD;
    size = 3;
    return ((uint32_t)(b0 & 0x0F) << 12) | ((uint32_t)(s[1] & 0x3F) << 6) | (s[2] & 0x3F);
  }
  if (b0 >= 0xF0 && b0 <= 0xF4) {
    uint8_t lo = b0 == 0xF0 ? 0x90 : 0x80, hi = b0 == 0xF4 ? 0x8F : 0xBF;
    if (!cont(1, lo, hi) || !cont(2, 0x80, 0xBF) || !cont(3, 0x80, 0xBF)) return 0xFFFD;
    size = 4;
    return ((uint32_t)(b0 & 0x07) << 18) | ((uint32_t)(s[1] & 0x3F) << 12) | ((uint32_t)(s[2] & 0x3F) << 6) |
           (s[3] & 0x3F);
  }
  return 0xFFFD;
}

int hexv(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// 4 hex digits at s[i..i+4) -> v; false if not hex (encoding/json getu4)
bool hex4(const uint8_t* s, size_t n, size_t i, uint32_t& v) {
  if (i + 4 > n) return false;
  v = 0;
  for (int k = 0; k < 4; k++) {
    int h = hexv(s[i + k]);
    if (h < 0) return false;
    v = (v << 4) | (uint32_t)h;
  }
  return true;
}

// first index at or after j (< n) whose byte is '"', '\\', < 0x20 or >= 0x80,
// 32 bytes per step; n if none
__attribute__((target("avx2"))) static size_t scan_plain_avx2(const uint8_t* s, size_t n, size_t j) {
  const __m256i quote = _mm256_set1_epi8('"'), bslash = _mm256_set1_epi8('\\'), c1f = _mm256_set1_epi8(0x1f);
  while (j + 32 <= n) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + j));
    // signed compare: bytes >= 0x80 are negative, so v <= 0x1f catches them and the control bytes
    __m256i hit = _mm256_or_si256(_mm256_cmpeq_epi8(v, quote), _mm256_cmpeq_epi8(v, bslash));
    hit = _mm256_or_si256(hit, _mm256_cmpgt_epi8(_mm256_add_epi8(c1f, _mm256_set1_epi8(1)), v));
    uint32_t m = (uint32_t)_mm256_movemask_epi8(hit);
    if (m) return j + (size_t)__builtin_ctz(m);
    j += 32;
  }
  return j;
}

static const bool g_avx2_scan = __builtin_cpu_supports("avx2");

struct Parser {
  const uint8_t* s;
  size_t n, i;
  JDoc* d;

  void ws() {
    while (i < n && is_ws(s[i])) i++;
  }

  // index of the first byte at or after j that is '"', '\\', < 0x20 or >= 0x80
  size_t scan_plain(size_t j) const {
    if (g_avx2_scan) {
      j = scan_plain_avx2(s, n, j);
      if (j + 32 <= n) return j;  // a hit inside a full block
    }
    const uint64_t ones = 0x0101010101010101ull, high = 0x8080808080808080ull;
    while (j + 8 <= n) {
      uint64_t v;
      memcpy(&v, s + j, 8);
      uint64_t q = v ^ (ones * '"'), b = v ^ (ones * '\\');
      uint64_t t = ((q - ones) & ~q) | ((b - ones) & ~b) | (v - ones * 0x20) | v;
      if (t & high) {  // a candidate in this word (borrows may flag false positives)
        for (size_t e = j + 8; j < e; j++) {
          uint8_t c = s[j];
          if (c == '"' || c == '\\' || c < 0x20 || c >= 0x80) return j;
        }
        continue;
      }
      j += 8;
    }
    while (j < n) {
      uint8_t c = s[j];
      if (c == '"' || c == '\\' || c < 0x20 || c >= 0x80) break;
      j++;
    }
    return j;
  }

  // string at s[i] == '"' -> J_STR node, unquoted as encoding/json unquoteBytes.
  // Plain strings (no escapes, ASCII) stay in the source text (bval = 1).
  bool string(uint32_t& node) {
    i++;
    size_t j0 = scan_plain(i);
    if (j0 < n && s[j0] == '"') {
      node = (uint32_t)d->nodes.size();
      d->nodes.push_back({J_STR, 1, (uint32_t)i, (uint32_t)(j0 - i)});
      i = j0 + 1;
      return true;
    }
    std::string& o = d->pool;
    uint32_t start = (uint32_t)o.size();
    while (true) {
      // bulk-copy the run of plain printable ASCII
      size_t j = scan_plain(i);
      if (j > i) o.append((const char*)s + i, j - i);
      i = j;
      if (i >= n) return false;
      uint8_t c = s[i];
      if (c == '"') {
        i++;
        break;
      }
      if (c < 0x20) return false;
      if (c >= 0x80) {  // coerce to well-formed UTF-8
        size_t sz;
        uint32_t r = decode_rune(s + i, n - i, sz);
        if (r == 0xFFFD && sz == 1)
          put_utf8(o, 0xFFFD);
        else
          o.append((const char*)s + i, sz);
        i += sz;
        continue;
      }
      // escape
      i++;
      if (i >= n) return false;
      uint8_t e = s[i++];
      switch (e) {
        case '"': o.push_back('"'); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(s, n, i, cp)) return false;
          i += 4;
          if (cp >= 0xD800 && cp < 0xE000) {
            uint32_t lo = 0;
            if (cp < 0xDC00 && i + 1 < n && s[i] == '\\' && s[i + 1] == 'u' && hex4(s, n, i + 2, lo) &&
                lo >= 0xDC00 && lo < 0xE000) {
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              i += 6;
            } else {
              cp = 0xFFFD;
            }
          }
          put_utf8(o, cp);
          break;
        }
        default:
          return false;
      }
    }
    node = (uint32_t)d->nodes.size();
    d->nodes.push_back({J_STR, 0, start, (uint32_t)(o.size() - start)});
    o.push_back('\0');
    return true;
  }

  bool number(uint32_t& node) {
    size_t j = i;
    if (j < n && s[j] == '-') j++;
    if (j < n && s[j] == '0') {
      j++;
    } else if (j < n && s[j] >= '1' && s[j] <= '9') {
      while (j < n && s[j] >= '0' && s[j] <= '9') j++;
    } else {
      return false;
    }
    if (j < n && s[j] == '.') {
      j++;
      if (!(j < n && s[j] >= '0' && s[j] <= '9')) return false;
      while (j < n && s[j] >= '0' && s[j] <= '9') j++;
    }
    if (j < n && (s[j] == 'e' || s[j] == 'E')) {
      j++;
      if (j < n && (s[j] == '+' || s[j] == '-')) j++;
      if (!(j < n && s[j] >= '0' && s[j] <= '9')) return false;
      while (j < n && s[j] >= '0' && s[j] <= '9') j++;
    }
    uint32_t start = (uint32_t)d->pool.size();
    d->pool.append((const char*)s + i, j - i);
    d->pool.push_back('\0');
    node = (uint32_t)d->nodes.size();
    d->nodes.push_back({J_NUM, 0, start, (uint32_t)(j - i)});
    i = j;
    return true;
  }

  // scalar value at s[i] (not a container)
  bool scalar(uint32_t& node) {
    uint8_t c = s[i];
    if (c == '"') return string(node);
    if (c == 'n' && i + 4 <= n && memcmp(s + i, "null", 4) == 0) {
      i += 4;
      node = (uint32_t)d->nodes.size();
      d->nodes.push_back({J_NULL, 0, 0, 0});
      return true;
    }
    if (c == 't' && i + 4 <= n && memcmp(s + i, "true", 4) == 0) {
      i += 4;
      node = (uint32_t)d->nodes.size();
      d->nodes.push_back({J_BOOL, 1, 0, 0});
      return true;
    }
    if (c == 'f' && i + 5 <= n && memcmp(s + i, "false", 5) == 0) {
      i += 5;
      node = (uint32_t)d->nodes.size();
      d->nodes.push_back({J_BOOL, 0, 0, 0});
      return true;
    }
    return number(node);
  }

  // frames: (tmp start << 1) | is_object
  bool run(uint32_t& root) {
    std::vector<uint64_t>& fr = d->frames;
    std::vector<uint32_t>& tmp = d->tmp;
    fr.clear();
    tmp.clear();
    uint32_t v = 0;
    // parse a value; containers push a frame and continue with their first member
  value:
    ws();
    if (i >= n) return false;
    if (s[i] == '{' || s[i] == '[') {
      bool obj = s[i] == '{';
      i++;
      if (fr.size() >= MAX_DEPTH) return false;
      fr.push_back(((uint64_t)tmp.size() << 1) | (obj ? 1u : 0u));
      ws();
      if (i < n && s[i] == (obj ? '}' : ']')) {
        i++;
        goto close;
      }
      if (obj) goto key;
      goto value;
    }
    if (!scalar(v)) return false;
    goto after;
  key:
    ws();
    if (i >= n || s[i] != '"') return false;
    {
      uint32_t k;
      if (!string(k)) return false;
      tmp.push_back(k);
    }
    ws();
    if (i >= n || s[i] != ':') return false;
    i++;
    goto value;
  close : {
    uint64_t f = fr.back();
    fr.pop_back();
    bool obj = f & 1;
    size_t t0 = (size_t)(f >> 1);
    v = (uint32_t)d->nodes.size();
    uint32_t cnt = (uint32_t)(tmp.size() - t0);
    d->nodes.push_back({obj ? J_OBJ : J_ARR, 0, (uint32_t)d->kids.size(), obj ? cnt / 2 : cnt});
    d->kids.insert(d->kids.end(), tmp.begin() + t0, tmp.end());
    tmp.resize(t0);
  }
  after:
    if (fr.empty()) {
      root = v;
      return true;
    }
    tmp.push_back(v);
    ws();
    if (i >= n) return false;
    {
      bool obj = fr.back() & 1;
      if (s[i] == ',') {
        i++;
        if (obj) goto key;
        goto value;
      }
      if (s[i] == (obj ? '}' : ']')) {
        i++;
        goto close;
      }
    }
    return false;
  }
};

int8_t B64_TAB[256];
struct B64Init {
  B64Init() {
    memset(B64_TAB, -1, sizeof(B64_TAB));
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int k = 0; k < 64; k++) B64_TAB[(uint8_t)a[k]] = (int8_t)k;
  }
} b64_init;

}  // namespace

bool JDoc::parse(const uint8_t* p, size_t n) {
  nodes.clear();
  kids.clear();
  pool.clear();
  src = p;
  Parser ps{p, n, 0, this};
  uint32_t root;
  if (!ps.run(root)) return false;
  ps.ws();
  if (ps.i != n) return false;
  return root == nodes.size() - 1;  // containers close after their children: the root is the last node
}

// encoding/json fold.go: foldFunc(name) picks equalFoldRight when the name holds
// k/K/s/S (the key may then spell them U+212A / U+017F), else ASCII case folding
// (asciiEqualFold == simpleLetterEqualFold on letter-only names).
bool go_key_matches(const char* key, size_t klen, const char* name, size_t nlen) {
  if (klen == nlen) {
    // equal lengths: a match can only be ASCII (U+017F / U+212A are multi-byte),
    // where every fold function reduces to ASCII case folding of the letters
    for (size_t k = 0; k < nlen; k++) {
      uint8_t sb = (uint8_t)name[k], tb = (uint8_t)key[k];
      if (sb == tb) continue;
      uint8_t su = sb & 0xDF;
      if (!(su >= 'A' && su <= 'Z') || su != (tb & 0xDF)) return false;
    }
    return true;
  }
  if (klen < nlen) return false;
  bool special = false;
  for (size_t k = 0; k < nlen; k++) {
    char c = name[k];
    special |= (c == 'k' || c == 'K' || c == 's' || c == 'S');
  }
  if (!special) return false;
  // equalFoldRight(name, key)
  const uint8_t* t = (const uint8_t*)key;
  size_t tl = klen;
  for (size_t k = 0; k < nlen; k++) {
    uint8_t sb = (uint8_t)name[k];
    if (tl == 0) return false;
    uint8_t tb = t[0];
    if (tb < 0x80) {
      if (sb != tb) {
        uint8_t su = sb & 0xDF;
        if (!(su >= 'A' && su <= 'Z') || su != (tb & 0xDF)) return false;
      }
      t++;
      tl--;
      continue;
    }
    size_t sz;
    uint32_t r = decode_rune(t, tl, sz);
    if (sb == 's' || sb == 'S') {
      if (r != 0x017F) return false;
    } else if (sb == 'k' || sb == 'K') {
      if (r != 0x212A) return false;
    } else {
      return false;
    }
    t += sz;
    tl -= sz;
  }
  return tl == 0;
}

int64_t JDoc::field(uint32_t obj, const char* name) const {
  const JNode& o = nodes[obj];
  if (o.type != J_OBJ) return -1;
  size_t nlen = strlen(name);
  int64_t found = -1;
  for (uint32_t k = 0; k < o.count; k++) {
    uint32_t key = kids[o.first + 2 * k];
    if (go_key_matches(str(key), nodes[key].count, name, nlen)) found = kids[o.first + 2 * k + 1];
  }
  return found;
}

namespace {

struct Merger {
  JDoc& d;

  uint32_t push(JNode n) {
    d.nodes.push_back(n);
    return (uint32_t)d.nodes.size() - 1;
  }
  uint32_t null_node() { return push({J_NULL, 0, 0, 0}); }
  uint32_t key_node(const char* name) {
    uint32_t off = (uint32_t)d.pool.size();
    d.pool.append(name);
    d.pool.push_back('\0');
    return push({J_STR, 0, off, (uint32_t)strlen(name)});
  }
  static int schema_len(const JField* s) {
    int n = 0;
    while (s && s[n].name) n++;
    return n;
  }

  // members of every object in occs (in order) as one object
  uint32_t merge(const std::vector<uint32_t>& occs, const JField* sch) {
    int nf = schema_len(sch);
    std::vector<uint32_t> pairs;
    std::vector<std::vector<uint32_t>> coll((size_t)nf);
    for (uint32_t o : occs) {
      const JNode on = d.nodes[o];
      for (uint32_t k = 0; k < on.count; k++) {
        uint32_t key = d.kids[on.first + 2 * k], val = d.kids[on.first + 2 * k + 1];
        int f = -1;
        for (int q = 0; q < nf && f < 0; q++)
          if (go_key_matches(d.str(key), d.nodes[key].count, sch[q].name, strlen(sch[q].name))) f = q;
        if (f < 0) {
          pairs.push_back(key);
          pairs.push_back(val);
        } else {
          coll[(size_t)f].push_back(val);
        }
      }
    }
    bool changed = occs.size() > 1;
    std::vector<uint32_t> res((size_t)nf, 0);
    for (int q = 0; q < nf; q++) {
      if (coll[(size_t)q].empty()) continue;
      res[(size_t)q] = sch[q].kind == JF_STRUCT ? rstruct(coll[(size_t)q], sch[q].sub)
                                                 : rslice(coll[(size_t)q], sch[q].sub);
      changed |= coll[(size_t)q].size() > 1 || res[(size_t)q] != coll[(size_t)q][0];
    }
    if (!changed) return occs[0];
    for (int q = 0; q < nf; q++) {
      if (coll[(size_t)q].empty()) continue;
      pairs.push_back(key_node(sch[q].name));
      pairs.push_back(res[(size_t)q]);
    }
    uint32_t first = (uint32_t)d.kids.size();
    d.kids.insert(d.kids.end(), pairs.begin(), pairs.end());
    return push({J_OBJ, 0, first, (uint32_t)(pairs.size() / 2)});
  }

  // *T field: the occurrences since the last null merge
  uint32_t rstruct(const std::vector<uint32_t>& vals, const JField* sub) {
    std::vector<uint32_t> cur;
    bool nil = true;
    for (uint32_t v : vals) {
      JType t = d.nodes[v].type;
      if (t == J_NULL) {
        cur.clear();
        nil = true;
      } else if (t == J_OBJ) {
        cur.push_back(v);
        nil = false;
      } else {
        return v;  // type error: reported by the typed decoder
      }
    }
    if (nil) return vals.size() == 1 ? vals[0] : null_node();
    return merge(cur, sub);
  }

  // []*T field: element slots survive truncation (see gojson.h)
  uint32_t rslice(const std::vector<uint32_t>& vals, const JField* sub) {
    struct Slot {
      bool nil = true;
      std::vector<uint32_t> occ;
    };
    std::vector<Slot> backing;
    size_t len = 0;
    bool nil = true;
    for (uint32_t v : vals) {
      JType t = d.nodes[v].type;
      if (t == J_NULL) {
        backing.clear();
        len = 0;
        nil = true;
        continue;
      }
      if (t != J_ARR) return v;
      nil = false;
      uint32_t n = d.len(v);
      size_t i = 0;
      for (; i < n; i++) {
        uint32_t e = d.elem(v, (uint32_t)i);
        if (i >= backing.size()) backing.emplace_back();
        if (i + 1 > len) len = i + 1;
        JType te = d.nodes[e].type;
        if (te == J_NULL) {
          backing[i] = Slot();
        } else if (te == J_OBJ) {
          backing[i].nil = false;
          backing[i].occ.push_back(e);
        } else {
          return e;
        }
      }
      if (i < len) len = i;
      if (i == 0) {
        backing.clear();
        len = 0;
      }
    }
    if (nil) return vals.size() == 1 ? vals[0] : null_node();
    std::vector<uint32_t> elems(len);
    bool changed = vals.size() > 1;
    for (size_t i = 0; i < len; i++) {
      if (backing[i].nil) {
        elems[i] = vals.size() == 1 ? d.elem(vals[0], (uint32_t)i) : null_node();
      } else {
        elems[i] = merge(backing[i].occ, sub);
        changed |= backing[i].occ.size() > 1 || elems[i] != backing[i].occ[0];
      }
    }
    if (!changed) return vals[0];
    uint32_t first = (uint32_t)d.kids.size();
    d.kids.insert(d.kids.end(), elems.begin(), elems.end());
    return push({J_ARR, 0, first, (uint32_t)len});
  }
};

}  // namespace

// false when merging obj under sch changes nothing: no schema field occurs
// twice, and none of the fields' values (struct, or a slice's object
// elements) needs merging itself -- the canonical encoder's output.  Merger
// then returns every node unchanged, so go_merge can skip it (and its
// allocations).
static bool needs_merge(const JDoc& d, uint32_t obj, const JField* sch) {
  int nf = 0;
  while (sch && sch[nf].name) nf++;
  if (!nf) return false;
  if (nf > 16) return true;
  uint8_t cnt[16] = {};
  uint32_t val[16] = {};
  const JNode& o = d.nodes[obj];
  for (uint32_t k = 0; k < o.count; k++) {
    uint32_t key = d.kids[o.first + 2 * k];
    for (int q = 0; q < nf; q++)
      if (go_key_matches(d.str(key), d.nodes[key].count, sch[q].name, strlen(sch[q].name))) {
        if (++cnt[q] > 1) return true;
        val[q] = d.kids[o.first + 2 * k + 1];
      }
  }
  for (int q = 0; q < nf; q++) {
    if (!cnt[q] || !sch[q].sub || !sch[q].sub[0].name) continue;
    const JNode& v = d.nodes[val[q]];
    if (sch[q].kind == JF_STRUCT) {
      if (v.type == J_OBJ && needs_merge(d, val[q], sch[q].sub)) return true;
    } else if (v.type == J_ARR) {
      for (uint32_t k = 0; k < v.count; k++) {
        uint32_t e = d.kids[v.first + k];
        if (d.nodes[e].type == J_OBJ && needs_merge(d, e, sch[q].sub)) return true;
      }
    }
  }
  return false;
}

void go_merge(JDoc& d, const JField* schema) {
  if (d.nodes.empty()) return;
  uint32_t root = d.root();
  if (d.at(root).type != J_OBJ) return;
  if (!needs_merge(d, root, schema)) return;
  Merger m{d};
  uint32_t r = m.merge({root}, schema);
  if (r != d.root()) {
    JNode copy = d.nodes[r];
    d.nodes.push_back(copy);  // root() is the last node
  }
}

bool b64_decode_append(const char* s, size_t n, std::vector<uint8_t>& out) {
  size_t base = out.size();
  out.resize(base + n / 4 * 3 + 3);
  uint8_t* w = out.data() + base;
  uint32_t q[4];
  int nq = 0;
  size_t k = 0;
  bool done = false;
  // fast path: whole quanta of alphabet characters
  while (k + 4 <= n) {
    int32_t a = B64_TAB[(uint8_t)s[k]], b = B64_TAB[(uint8_t)s[k + 1]], c = B64_TAB[(uint8_t)s[k + 2]],
            e = B64_TAB[(uint8_t)s[k + 3]];
    if ((a | b | c | e) < 0) break;
    uint32_t v = ((uint32_t)a << 18) | ((uint32_t)b << 12) | ((uint32_t)c << 6) | (uint32_t)e;
    w[0] = (uint8_t)(v >> 16);
    w[1] = (uint8_t)(v >> 8);
    w[2] = (uint8_t)v;
    w += 3;
    k += 4;
  }
  for (; k < n; k++) {
    uint8_t c = (uint8_t)s[k];
    if (c == '\r' || c == '\n') continue;
    if (c == '=') {
      // padding: quantum position 2 needs "==", position 3 one '='; then only newlines may follow
      if (nq < 2) return false;
      if (nq == 2) {
        size_t m = k + 1;
        while (m < n && (s[m] == '\r' || s[m] == '\n')) m++;
        if (m >= n || s[m] != '=') return false;
        k = m;
      }
      done = true;
      k++;
      break;
    }
    int8_t v = B64_TAB[c];
    if (v < 0) return false;
    q[nq++] = (uint32_t)v;
    if (nq == 4) {
      uint32_t a = (q[0] << 18) | (q[1] << 12) | (q[2] << 6) | q[3];
      w[0] = (uint8_t)(a >> 16);
      w[1] = (uint8_t)(a >> 8);
      w[2] = (uint8_t)a;
      w += 3;
      nq = 0;
    }
  }
  if (done) {
    for (; k < n; k++)
      if (s[k] != '\r' && s[k] != '\n') return false;
    uint32_t a = (q[0] << 18) | (q[1] << 12) | (nq == 3 ? q[2] << 6 : 0);
    *w++ = (uint8_t)(a >> 16);
    if (nq == 3) *w++ = (uint8_t)(a >> 8);
  } else if (nq != 0) {
    return false;  // unpadded tail
  }
  out.resize((size_t)(w - out.data()));
  return true;
}

// 32 alphabet characters -> 24 bytes at w (32 bytes written; the caller keeps
// 8 bytes of slack), AVX2 nibble-table validation and shift-merge (Mula &
// Lemire, "Faster Base64 Encoding and Decoding Using AVX2 Instructions").
// false: some character is outside the standard alphabet (the scalar code
// then decides).
__attribute__((target("avx2"))) static bool b64_block32_avx2(const char* s, uint8_t* w) {
  const __m256i in = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s));
  const __m256i lut_lo = _mm256_setr_epi8(0x15, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x13, 0x1A, 0x1B,
                                          0x1B, 0x1B, 0x1A, 0x15, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11, 0x11,
                                          0x13, 0x1A, 0x1B, 0x1B, 0x1B, 0x1A);
  const __m256i lut_hi = _mm256_setr_epi8(0x10, 0x10, 0x01, 0x02, 0x04, 0x08, 0x04, 0x08, 0x10, 0x10, 0x10, 0x10, 0x10,
                                          0x10, 0x10, 0x10, 0x10, 0x10, 0x01, 0x02, 0x04, 0x08, 0x04, 0x08, 0x10, 0x10,
                                          0x10, 0x10, 0x10, 0x10, 0x10, 0x10);
  const __m256i lut_roll = _mm256_setr_epi8(0, 16, 19, 4, -65, -65, -71, -71, 0, 0, 0, 0, 0, 0, 0, 0, 0, 16, 19, 4, -65,
                                            -65, -71, -71, 0, 0, 0, 0, 0, 0, 0, 0);
  const __m256i m2f = _mm256_set1_epi8(0x2f);
  const __m256i hi_n = _mm256_and_si256(_mm256_srli_epi32(in, 4), m2f);
  const __m256i lo_n = _mm256_and_si256(in, m2f);
  const __m256i lo = _mm256_shuffle_epi8(lut_lo, lo_n);
  const __m256i hi = _mm256_shuffle_epi8(lut_hi, hi_n);
  if (!_mm256_testz_si256(lo, hi)) return false;
  const __m256i roll = _mm256_shuffle_epi8(lut_roll, _mm256_add_epi8(_mm256_cmpeq_epi8(in, m2f), hi_n));
  const __m256i v = _mm256_add_epi8(in, roll);
  const __m256i ab = _mm256_maddubs_epi16(v, _mm256_set1_epi32(0x01400140));
  __m256i o = _mm256_madd_epi16(ab, _mm256_set1_epi32(0x00011000));
  o = _mm256_shuffle_epi8(o, _mm256_setr_epi8(2, 1, 0, 6, 5, 4, 10, 9, 8, 14, 13, 12, -1, -1, -1, -1, 2, 1, 0, 6, 5, 4,
                                              10, 9, 8, 14, 13, 12, -1, -1, -1, -1));
  o = _mm256_permutevar8x32_epi32(o, _mm256_setr_epi32(0, 1, 2, 4, 5, 6, 7, 7));
  _mm256_storeu_si256(reinterpret_cast<__m256i*>(w), o);
  return true;
}

static const bool g_avx2 = __builtin_cpu_supports("avx2");

bool b64_decode_strict_append(const char* s, size_t n, std::vector<uint8_t>& out) {
  if (n % 4) return false;
  size_t base = out.size();
  out.resize(base + n / 4 * 3 + 8);  // + slack for the 32-byte stores of the vector blocks
  uint8_t* w = out.data() + base;
  size_t k = 0;
  if (g_avx2)
    for (; k + 32 < n; k += 32) {  // whole 32-character blocks before the last quantum
      if (!b64_block32_avx2(s + k, w)) return false;
      w += 24;
    }
  for (; k + 4 < n; k += 4) {  // every quantum but the last: 4 alphabet characters
    int32_t a = B64_TAB[(uint8_t)s[k]], b = B64_TAB[(uint8_t)s[k + 1]], c = B64_TAB[(uint8_t)s[k + 2]],
            e = B64_TAB[(uint8_t)s[k + 3]];
    if ((a | b | c | e) < 0) return false;
    uint32_t v = ((uint32_t)a << 18) | ((uint32_t)b << 12) | ((uint32_t)c << 6) | (uint32_t)e;
    w[0] = (uint8_t)(v >> 16);
    w[1] = (uint8_t)(v >> 8);
    w[2] = (uint8_t)v;
    w += 3;
  }
  if (n) {  // last quantum: "xxxx", "xxx=" or "xx=="
    int pad = s[n - 1] == '=' ? (s[n - 2] == '=' ? 2 : 1) : 0;
    int32_t a = B64_TAB[(uint8_t)s[k]], b = B64_TAB[(uint8_t)s[k + 1]];
    int32_t c = pad == 2 ? 0 : B64_TAB[(uint8_t)s[k + 2]], e = pad ? 0 : B64_TAB[(uint8_t)s[k + 3]];
    if ((a | b | c | e) < 0) return false;
    uint32_t v = ((uint32_t)a << 18) | ((uint32_t)b << 12) | ((uint32_t)c << 6) | (uint32_t)e;
    w[0] = (uint8_t)(v >> 16);
    if (pad < 2) w[1] = (uint8_t)(v >> 8);
    if (pad < 1) w[2] = (uint8_t)v;
    w += 3 - pad;
  }
  out.resize((size_t)(w - out.data()));
  return true;
}

bool b64_decode(const char* s, size_t n, std::vector<uint8_t>& out) {
  out.clear();
  return b64_decode_append(s, n, out);
}

void b64_encode(const uint8_t* p, size_t n, std::string& out) {
  static const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  size_t k = 0;
  for (; k + 3 <= n; k += 3) {
    uint32_t v = ((uint32_t)p[k] << 16) | ((uint32_t)p[k + 1] << 8) | p[k + 2];
    out.push_back(a[v >> 18]);
    out.push_back(a[(v >> 12) & 63]);
    out.push_back(a[(v >> 6) & 63]);
    out.push_back(a[v & 63]);
  }
  if (n - k == 1) {
    uint32_t v = (uint32_t)p[k] << 16;
    out.push_back(a[v >> 18]);
    out.push_back(a[(v >> 12) & 63]);
    out += "==";
  } else if (n - k == 2) {
    uint32_t v = ((uint32_t)p[k] << 16) | ((uint32_t)p[k + 1] << 8);
    out.push_back(a[v >> 18]);
    out.push_back(a[(v >> 12) & 63]);
    out.push_back(a[(v >> 6) & 63]);
    out.push_back('=');
  }
}

DecStatus dec_bytes(const JDoc& d, int64_t node, std::vector<uint8_t>& out) {
  out.clear();
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return D_NIL;
  if (d.at((uint32_t)node).type != J_STR) return D_ERR;
  const char* s = d.str((uint32_t)node);
  size_t n = d.len((uint32_t)node);
  // canonical text (the Go encoder's output) through the vector decoder, anything
  // else through the lenient one: same bytes where both accept
  if (b64_decode_strict_append(s, n, out)) return D_OK;
  if (!b64_decode(s, n, out)) return D_ERR;
  return D_OK;
}

DecStatus dec_int(const JDoc& d, int64_t node, int64_t& out) {
  out = 0;
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return D_NIL;
  if (d.at((uint32_t)node).type != J_NUM) return D_ERR;
  const char* t = d.str((uint32_t)node);
  uint32_t L = d.len((uint32_t)node);
  bool negv = false;
  uint32_t k = 0;
  if (t[0] == '-') {
    negv = true;
    k = 1;
  }
  unsigned __int128 v = 0;
  for (; k < L; k++) {
    if (t[k] < '0' || t[k] > '9') return D_ERR;  // fraction / exponent: not an int
    v = v * 10 + (uint32_t)(t[k] - '0');
    if (v > ((unsigned __int128)1 << 64)) return D_ERR;
  }
  if (negv) {
    if (v > ((unsigned __int128)1 << 63)) return D_ERR;
    out = -(int64_t)(uint64_t)v;
  } else {
    if (v >= ((unsigned __int128)1 << 63)) return D_ERR;
    out = (int64_t)v;
  }
  return D_OK;
}

DecStatus dec_string(const JDoc& d, int64_t node, std::string& out) {
  out.clear();
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return D_NIL;
  if (d.at((uint32_t)node).type != J_STR) return D_ERR;
  out.assign(d.str((uint32_t)node), d.len((uint32_t)node));
  return D_OK;
}

// curve and element of a mathlib element object; D_OK / D_NIL / D_ERR / D_PANIC
static DecStatus elem_fields(const JDoc& d, int64_t node, int64_t& elem) {
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return D_NIL;
  if (d.at((uint32_t)node).type != J_OBJ) return D_ERR;
  int64_t curve = 0;
  if (dec_int(d, d.field((uint32_t)node, "curve"), curve) == D_ERR) return D_ERR;
  elem = d.field((uint32_t)node, "element");
  if (elem >= 0 && d.at((uint32_t)elem).type != J_NULL && d.at((uint32_t)elem).type != J_STR) return D_ERR;
  return curve == 1 ? D_OK : D_PANIC;
}

DecStatus dec_bytes_append(const JDoc& d, int64_t node, std::vector<uint8_t>& out) {
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) return D_NIL;
  if (d.at((uint32_t)node).type != J_STR) return D_ERR;
  const char* s = d.str((uint32_t)node);
  size_t n = d.len((uint32_t)node), mark = out.size();
  if (b64_decode_strict_append(s, n, out)) return D_OK;
  out.resize(mark);  // the strict decoder may have stopped part way
  if (!b64_decode_append(s, n, out)) {
    out.resize(mark);
    return D_ERR;
  }
  return D_OK;
}

DecStatus dec_elem_append(const JDoc& d, int64_t node, std::vector<uint8_t>& out) {
  int64_t el = -1;
  DecStatus st = elem_fields(d, node, el);
  if (st == D_NIL || st == D_ERR) return st;
  return dec_bytes_append(d, el, out) == D_ERR ? D_ERR : st;
}

ElemBytes dec_elem(const JDoc& d, int64_t node) {
  ElemBytes r;
  int64_t el = -1;
  r.st = elem_fields(d, node, el);
  if (r.st == D_NIL || r.st == D_ERR) return r;
  DecStatus bs = dec_bytes(d, el, r.raw);
  if (bs == D_ERR) r.st = D_ERR;  // a bad element string fails Unmarshal before the curve id is used
  return r;
}

DecStatus dec_elem_into(const JDoc& d, int64_t node, std::vector<uint8_t>& dst, size_t& off, uint32_t& len) {
  int64_t el = -1;
  DecStatus st = elem_fields(d, node, el);
  if (st == D_NIL || st == D_ERR) return st;
  size_t mark = dst.size();
  size_t a = (mark + 15) & ~(size_t)15;
  dst.resize(a, 0);
  if (el >= 0 && d.at((uint32_t)el).type == J_STR &&
      !b64_decode_append(d.str((uint32_t)el), d.len((uint32_t)el), dst)) {
    dst.resize(mark);
    return D_ERR;
  }
  if (st == D_PANIC) {
    dst.resize(mark);
    return D_PANIC;
  }
  off = a;
  len = (uint32_t)(dst.size() - a);
  return D_OK;
}

}  // namespace ftsh
