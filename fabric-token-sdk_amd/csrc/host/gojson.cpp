#include "gojson.h"

#include <string.h>

namespace ftsh {

namespace {

struct Parser {
  const uint8_t* s;
  size_t n, i;
  JDoc* d;
  int depth;

  void ws() {
    while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\r' || s[i] == '\n')) i++;
  }

  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) {
      o.push_back((char)cp);
    } else if (cp < 0x800) {
      o.push_back((char)(0xC0 | (cp >> 6)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      o.push_back((char)(0xE0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      o.push_back((char)(0xF0 | (cp >> 18)));
      o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }

  static int hexv(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }

  bool hex4(uint32_t& v) {
    if (i + 4 > n) return false;
    v = 0;
    for (int k = 0; k < 4; k++) {
      int h = hexv(s[i + k]);
      if (h < 0) return false;
      v = (v << 4) | (uint32_t)h;
    }
    i += 4;
    return true;
  }

  // parses a string starting at s[i] == '"', appends to pool; returns node index
  bool string(uint32_t& node) {
    i++;
    uint32_t start = (uint32_t)d->pool.size();
    std::string& o = d->pool;
    while (true) {
      if (i >= n) return false;
      uint8_t c = s[i];
      if (c == '"') {
        i++;
        break;
      }
      if (c == '\\') {
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
            if (!hex4(cp)) return false;
            if (cp >= 0xD800 && cp < 0xDC00) {
              uint32_t lo = 0;
              size_t save = i;
              if (i + 1 < n && s[i] == '\\' && s[i + 1] == 'u') {
                i += 2;
                if (hex4(lo) && lo >= 0xDC00 && lo < 0xE000) {
                  cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                } else {
                  i = save;
                  cp = 0xFFFD;
                }
              } else {
                cp = 0xFFFD;
              }
            } else if (cp >= 0xD800 && cp < 0xE000) {
              cp = 0xFFFD;
            }
            put_utf8(o, cp);
            break;
          }
          default:
            return false;
        }
        continue;
      }
      if (c < 0x20) return false;
      o.push_back((char)c);
      i++;
    }
    node = (uint32_t)d->nodes.size();
    d->nodes.push_back({J_STR, 0, start, (uint32_t)(d->pool.size() - start)});
    d->pool.push_back('\0');
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

  bool value(uint32_t& node) {
    if (++depth > 10000) return false;
    ws();
    if (i >= n) return false;
    uint8_t c = s[i];
    bool ok;
    if (c == '{') {
      ok = object(node);
    } else if (c == '[') {
      ok = array(node);
    } else if (c == '"') {
      ok = string(node);
    } else if (c == 'n' && i + 4 <= n && memcmp(s + i, "null", 4) == 0) {
      i += 4;
      node = (uint32_t)d->nodes.size();
      d->nodes.push_back({J_NULL, 0, 0, 0});
      ok = true;
    } else if (c == 't' && i + 4 <= n && memcmp(s + i, "true", 4) == 0) {
      i += 4;
      node = (uint32_t)d->nodes.size();
      d->nodes.push_back({J_BOOL, 1, 0, 0});
      ok = true;
    } else if (c == 'f' && i + 5 <= n && memcmp(s + i, "false", 5) == 0) {
      i += 5;
      node = (uint32_t)d->nodes.size();
      d->nodes.push_back({J_BOOL, 0, 0, 0});
      ok = true;
    } else {
      ok = number(node);
    }
    depth--;
    return ok;
  }

  bool object(uint32_t& node) {
    i++;
    std::vector<uint32_t> tmp;
    ws();
    if (i < n && s[i] == '}') {
      i++;
    } else {
      while (true) {
        ws();
        if (i >= n || s[i] != '"') return false;
        uint32_t k, v;
        if (!string(k)) return false;
        ws();
        if (i >= n || s[i] != ':') return false;
        i++;
        if (!value(v)) return false;
        tmp.push_back(k);
        tmp.push_back(v);
        ws();
        if (i >= n) return false;
        if (s[i] == ',') {
          i++;
          continue;
        }
        if (s[i] == '}') {
          i++;
          break;
        }
        return false;
      }
    }
    node = (uint32_t)d->nodes.size();
    d->nodes.push_back({J_OBJ, 0, (uint32_t)d->kids.size(), (uint32_t)(tmp.size() / 2)});
    d->kids.insert(d->kids.end(), tmp.begin(), tmp.end());
    return true;
  }

  bool array(uint32_t& node) {
    i++;
    std::vector<uint32_t> tmp;
    ws();
    if (i < n && s[i] == ']') {
      i++;
    } else {
      while (true) {
        uint32_t v;
        if (!value(v)) return false;
        tmp.push_back(v);
        ws();
        if (i >= n) return false;
        if (s[i] == ',') {
          i++;
          continue;
        }
        if (s[i] == ']') {
          i++;
          break;
        }
        return false;
      }
    }
    node = (uint32_t)d->nodes.size();
    d->nodes.push_back({J_ARR, 0, (uint32_t)d->kids.size(), (uint32_t)tmp.size()});
    d->kids.insert(d->kids.end(), tmp.begin(), tmp.end());
    return true;
  }
};

// ASCII-only case fold (Go's EqualFold on ASCII field names)
bool fold_eq(const char* a, uint32_t alen, const char* b) {
  size_t blen = strlen(b);
  if (alen != blen) return false;
  for (uint32_t k = 0; k < alen; k++) {
    char x = a[k], y = b[k];
    if (x >= 'A' && x <= 'Z') x += 32;
    if (y >= 'A' && y <= 'Z') y += 32;
    if (x != y) return false;
  }
  return true;
}

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
  nodes.reserve(n / 8 + 8);
  pool.reserve(n);
  Parser ps{p, n, 0, this, 0};
  uint32_t root;
  if (!ps.value(root)) return false;
  ps.ws();
  if (ps.i != n) return false;
  // root must be the last node pushed; move it to index 0 by convention
  if (root != nodes.size() - 1) return false;
  return true;
}

int64_t JDoc::field(uint32_t obj, const char* name) const {
  const JNode& o = nodes[obj];
  if (o.type != J_OBJ) return -1;
  int64_t found = -1;
  for (uint32_t k = 0; k < o.count; k++) {
    uint32_t key = kids[o.first + 2 * k];
    if (fold_eq(str(key), nodes[key].count, name)) found = kids[o.first + 2 * k + 1];
  }
  return found;
}

bool b64_decode(const char* s, size_t n, std::vector<uint8_t>& out) {
  out.clear();
  std::string t;
  t.reserve(n);
  for (size_t k = 0; k < n; k++)
    if (s[k] != '\r' && s[k] != '\n') t.push_back(s[k]);
  if (t.size() % 4 != 0) return false;
  out.reserve(t.size() / 4 * 3);
  for (size_t q = 0; q < t.size(); q += 4) {
    bool last = q + 4 == t.size();
    int pad = 0;
    if (t[q + 3] == '=') {
      if (!last) return false;
      pad = (t[q + 2] == '=') ? 2 : 1;
    }
    uint32_t acc = 0;
    for (int k = 0; k < 4 - pad; k++) {
      int8_t v = B64_TAB[(uint8_t)t[q + k]];
      if (v < 0) return false;
      acc = (acc << 6) | (uint32_t)v;
    }
    acc <<= 6 * pad;
    out.push_back((uint8_t)(acc >> 16));
    if (pad < 2) out.push_back((uint8_t)(acc >> 8));
    if (pad < 1) out.push_back((uint8_t)acc);
  }
  return true;
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
  if (!b64_decode(d.str((uint32_t)node), d.len((uint32_t)node), out)) return D_ERR;
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

ElemBytes dec_elem(const JDoc& d, int64_t node) {
  ElemBytes r;
  if (node < 0 || d.at((uint32_t)node).type == J_NULL) {
    r.st = D_NIL;
    return r;
  }
  if (d.at((uint32_t)node).type != J_OBJ) {
    r.st = D_ERR;
    return r;
  }
  int64_t curve = 0;
  DecStatus cs = dec_int(d, d.field((uint32_t)node, "curve"), curve);
  if (cs == D_ERR) {
    r.st = D_ERR;
    return r;
  }
  DecStatus bs = dec_bytes(d, d.field((uint32_t)node, "element"), r.raw);
  if (bs == D_ERR) {
    r.st = D_ERR;
    return r;
  }
  if (curve != 1) {
    r.st = D_PANIC;
    return r;
  }
  r.st = D_OK;
  return r;
}

}  // namespace ftsh
