"""Go ``encoding/json`` restated for the zkatdlog wire format (TEST INFRASTRUCTURE ONLY).

Encoding follows ``json.Marshal``: struct fields in declaration order, no
whitespace, ``[]byte`` as standard base64 with padding, nil slices/pointers as
``null``, HTML-safe string escaping.  mathlib's G1/G2/Zr elements marshal as
``{"curve":<CurveID>,"element":<base64(Bytes())>}`` ([EXT]).

Decoding follows ``json.Unmarshal`` of Go 1.18 (reference go.mod:3): object
keys match struct fields exactly, else by encoding/json fold.go's foldFunc
for the field name (ASCII case folding; when the name holds k/K/s/S the key
may also spell them U+212A KELVIN SIGN / U+017F LATIN SMALL LETTER LONG S),
unknown keys are ignored, a later duplicate overwrites an earlier leaf value
and merges into an earlier struct / slice-of-struct value (resolve()),
``null`` leaves a nil pointer/slice, strings are unquoted as unquoteBytes does
(invalid UTF-8 bytes and unpaired surrogates become U+FFFD, one per byte),
``[]byte`` is decoded by ``base64.StdEncoding`` (``\\r``/``\\n`` ignored,
padding required).
"""
import base64
import json

BN254 = 1


class GoJSONError(Exception):
    pass


# ------------------------------------------------------------------ encoding
def enc_str(s):
    out = json.dumps(s, ensure_ascii=False)
    return (out.replace("<", "\\u003c").replace(">", "\\u003e")
            .replace("&", "\\u0026").replace("\u2028", "\\u2028").replace("\u2029", "\\u2029"))


def enc_bytes(b):
    if b is None:
        return "null"
    return '"' + base64.b64encode(bytes(b)).decode() + '"'


def enc_elem(raw, curve=BN254):
    """mathlib curveElement{CurveID `json:"curve"`, ElementBytes `json:"element"`}."""
    if raw is None:
        return "null"
    return '{"curve":%d,"element":%s}' % (curve, enc_bytes(raw))


def enc_list(items, f):
    if items is None:
        return "null"
    return "[" + ",".join(f(x) for x in items) + "]"


def enc_struct(fields):
    """fields: list of (name, already-encoded json text)."""
    return "{" + ",".join(enc_str(k) + ":" + v for k, v in fields) + "}"


# ------------------------------------------------------------------ decoding
def _decode_rune(b, i):
    """unicode/utf8.DecodeRune on bytes b at i -> (rune, size); invalid -> (0xFFFD, 1)."""
    n = len(b)
    b0 = b[i]
    if b0 < 0x80:
        return b0, 1

    def cont(k, lo=0x80, hi=0xBF):
        return i + k < n and lo <= b[i + k] <= hi
    if 0xC2 <= b0 <= 0xDF:
        if cont(1):
            return ((b0 & 0x1F) << 6) | (b[i + 1] & 0x3F), 2
        return 0xFFFD, 1
    if 0xE0 <= b0 <= 0xEF:
        lo = 0xA0 if b0 == 0xE0 else 0x80
        hi = 0x9F if b0 == 0xED else 0xBF
        if cont(1, lo, hi) and cont(2):
            return ((b0 & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F), 3
        return 0xFFFD, 1
    if 0xF0 <= b0 <= 0xF4:
        lo = 0x90 if b0 == 0xF0 else 0x80
        hi = 0x8F if b0 == 0xF4 else 0xBF
        if cont(1, lo, hi) and cont(2) and cont(3):
            return (((b0 & 0x07) << 18) | ((b[i + 1] & 0x3F) << 12) | ((b[i + 2] & 0x3F) << 6)
                    | (b[i + 3] & 0x3F)), 4
        return 0xFFFD, 1
    return 0xFFFD, 1


_HEX = b"0123456789abcdefABCDEF"
_WS = b" \t\r\n"
MAX_DEPTH = 10000  # encoding/json scanner.go maxNestingDepth


class _Parser:
    """RFC 8259 parser over BYTES (as encoding/json's scanner) that keeps object
    members as an ordered list of (key, value) pairs, so duplicate keys survive
    to the typed decoder.  Strings come out unquoted as Go's unquoteBytes."""

    def __init__(self, text):
        if isinstance(text, str):
            text = text.encode("utf-8")
        self.s = bytes(text)
        self.i = 0
        self.depth = 0

    def ws(self):
        s, i = self.s, self.i
        while i < len(s) and s[i] in _WS:
            i += 1
        self.i = i

    def parse(self):
        self.ws()
        v = self.value()
        self.ws()
        if self.i != len(self.s):
            raise GoJSONError("invalid character after top-level value")
        return v

    def value(self):
        self.ws()
        if self.i >= len(self.s):
            raise GoJSONError("unexpected end of JSON input")
        c = self.s[self.i]
        if c in b"{[":
            self.depth += 1
            if self.depth > MAX_DEPTH:
                raise GoJSONError("exceeded max depth")
            v = self.obj() if c == ord("{") else self.arr()
            self.depth -= 1
            return v
        if c == ord('"'):
            return ("str", self.string())
        if self.s.startswith(b"null", self.i):
            self.i += 4
            return ("null", None)
        if self.s.startswith(b"true", self.i):
            self.i += 4
            return ("bool", True)
        if self.s.startswith(b"false", self.i):
            self.i += 5
            return ("bool", False)
        return self.number()

    def obj(self):
        self.i += 1
        pairs = []
        self.ws()
        if self.i < len(self.s) and self.s[self.i] == ord("}"):
            self.i += 1
            return ("obj", pairs)
        while True:
            self.ws()
            if self.i >= len(self.s) or self.s[self.i] != ord('"'):
                raise GoJSONError("expected object key")
            k = self.string()
            self.ws()
            if self.i >= len(self.s) or self.s[self.i] != ord(":"):
                raise GoJSONError("expected ':'")
            self.i += 1
            v = self.value()
            pairs.append((k, v))
            self.ws()
            if self.i >= len(self.s):
                raise GoJSONError("unexpected end")
            if self.s[self.i] == ord(","):
                self.i += 1
                continue
            if self.s[self.i] == ord("}"):
                self.i += 1
                return ("obj", pairs)
            raise GoJSONError("expected ',' or '}'")

    def arr(self):
        self.i += 1
        items = []
        self.ws()
        if self.i < len(self.s) and self.s[self.i] == ord("]"):
            self.i += 1
            return ("arr", items)
        while True:
            items.append(self.value())
            self.ws()
            if self.i >= len(self.s):
                raise GoJSONError("unexpected end")
            if self.s[self.i] == ord(","):
                self.i += 1
                continue
            if self.s[self.i] == ord("]"):
                self.i += 1
                return ("arr", items)
            raise GoJSONError("expected ',' or ']'")

    def _u4(self, i):
        h = self.s[i:i + 4]
        if len(h) != 4 or any(ch not in _HEX for ch in h):
            return None
        return int(h, 16)

    def string(self):
        s = self.s
        i = self.i + 1
        out = []
        esc = {ord('"'): '"', ord("\\"): "\\", ord("/"): "/", ord("b"): "\b", ord("f"): "\f",
               ord("n"): "\n", ord("r"): "\r", ord("t"): "\t"}
        while True:
            if i >= len(s):
                raise GoJSONError("unterminated string")
            c = s[i]
            if c == ord('"'):
                self.i = i + 1
                return "".join(out)
            if c == ord("\\"):
                i += 1
                if i >= len(s):
                    raise GoJSONError("bad escape")
                e = s[i]
                if e in esc:
                    out.append(esc[e])
                    i += 1
                elif e == ord("u"):
                    cp = self._u4(i + 1)
                    if cp is None:
                        raise GoJSONError("bad \\u escape")
                    i += 5
                    if 0xD800 <= cp < 0xE000:
                        lo = self._u4(i + 2) if s[i:i + 2] == b"\\u" else None
                        if cp < 0xDC00 and lo is not None and 0xDC00 <= lo < 0xE000:
                            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00)
                            i += 6
                        else:
                            cp = 0xFFFD
                    out.append(chr(cp))
                else:
                    raise GoJSONError("bad escape")
                continue
            if c < 0x20:
                raise GoJSONError("control character in string")
            if c < 0x80:
                out.append(chr(c))
                i += 1
                continue
            r, size = _decode_rune(s, i)
            out.append(chr(r))
            i += size

    def number(self):
        s = self.s
        j = self.i
        dig = b"0123456789"
        if j < len(s) and s[j] == ord("-"):
            j += 1
        if j < len(s) and s[j] == ord("0"):
            j += 1
        elif j < len(s) and s[j] in dig:
            while j < len(s) and s[j] in dig:
                j += 1
        else:
            raise GoJSONError("invalid character")
        if j < len(s) and s[j] == ord("."):
            j += 1
            if not (j < len(s) and s[j] in dig):
                raise GoJSONError("bad number")
            while j < len(s) and s[j] in dig:
                j += 1
        if j < len(s) and s[j] in b"eE":
            j += 1
            if j < len(s) and s[j] in b"+-":
                j += 1
            if not (j < len(s) and s[j] in dig):
                raise GoJSONError("bad number")
            while j < len(s) and s[j] in dig:
                j += 1
        tok = s[self.i:j].decode()
        self.i = j
        return ("num", tok)


def parse(text):
    return _Parser(text).parse()


def key_matches(key, name):
    """encoding/json: key selects the struct field ``name`` (ASCII) when equal,
    else under foldFunc(name): every name letter matches the same letter in
    either ASCII case, and -- only for names holding k/K/s/S (equalFoldRight) --
    s/S also matches U+017F and k/K matches U+212A."""
    if key == name:
        return True
    special = any(ch in "kKsS" for ch in name)
    if len(key) != len(name):
        return False
    for kc, nc in zip(key, name):
        if kc == nc:
            continue
        if nc.isascii() and nc.isalpha() and kc.isascii() and kc.lower() == nc.lower():
            continue
        if special and nc in "sS" and kc == "\u017f":
            continue
        if special and nc in "kK" and kc == "\u212a":
            continue
        return False
    return True


def field(obj, name):
    """Go struct-field lookup: the LAST member whose key selects ``name``
    (key_matches; Go applies members in order, so the last wins).  Returns None
    when the key is absent (zero value)."""
    if obj[0] != "obj":
        raise GoJSONError("cannot unmarshal %s into struct" % obj[0])
    found = None
    for k, v in obj[1]:
        if key_matches(k, name):
            found = v
    return found


# ------------------------------------------------------------------ duplicate keys
# Go 1.18 decode.go does not REPLACE a struct-pointer or slice-of-struct-pointer
# field when its key occurs again, it decodes INTO the value already there:
#   * indirect() keeps a non-nil pointer and object() does not zero the struct,
#     so two objects for one *T field merge key by key (a null in between resets
#     the pointer to nil);
#   * array() decodes element i into the slice's existing element i (a non-nil
#     *T element again merges), then truncates to the new length; the backing
#     array survives the truncation, so a later, longer array re-exposes (and
#     merges into) the old elements -- growth copies every element below the
#     write index, so nothing reachable is ever dropped; an empty JSON array
#     installs a fresh empty slice, null a nil one.
# Leaf fields ([]byte, string, int, mathlib elements with their own
# UnmarshalJSON) are replaced, which field()'s last-match lookup already gives.
# resolve() rewrites a parsed value so that every struct-typed field named in
# `schema` appears once, holding the merged value; schema = {FieldName:
# (STRUCT | SLICE, sub_schema)}.
STRUCT, SLICE = "struct", "slice"
NULL = ("null", None)


def resolve(v, schema):
    """v: a parsed top-level value decoded into a fresh struct."""
    if v is None or v[0] != "obj" or not schema:
        return v
    return _merge([v], schema)


def _merge(occs, schema):
    pairs, coll = [], {}
    for o in occs:
        for k, val in o[1]:
            f = next((n for n in schema if key_matches(k, n)), None)
            if f is None:
                pairs.append((k, val))
            else:
                coll.setdefault(f, []).append(val)
    for f, vals in coll.items():
        kind, sub = schema[f]
        pairs.append((f, _res_struct(vals, sub) if kind == STRUCT else _res_slice(vals, sub)))
    return ("obj", pairs)


def _res_struct(vals, sub):
    cur = None
    for val in vals:
        if val[0] == "null":
            cur = None
        elif val[0] == "obj":
            cur = (cur or []) + [val]
        else:
            return val  # type error: Unmarshal fails whatever follows; the decoder reports it
    return NULL if cur is None else _merge(cur, sub)


def _res_slice(vals, sub):
    backing, ln, isnil = [], 0, True
    for val in vals:
        if val[0] == "null":
            backing, ln, isnil = [], 0, True
            continue
        if val[0] != "arr":
            return val
        isnil = False
        i = 0
        for e in val[1]:
            if i >= len(backing):
                backing.append(None)
            ln = max(ln, i + 1)
            if e[0] == "null":
                backing[i] = None
            elif e[0] == "obj":
                backing[i] = (backing[i] or []) + [e]
            else:
                return e
            i += 1
        ln = i if i < ln else ln
        if i == 0:
            backing, ln = [], 0
    if isnil:
        return NULL
    return ("arr", [NULL if s is None else _merge(s, sub) for s in backing[:ln]])


def b64_std_decode(s):
    """Go base64.StdEncoding.DecodeString: '\\r' and '\\n' are skipped,
    padding is mandatory, trailing bits may be non-zero."""
    s = s.replace("\r", "").replace("\n", "")
    if len(s) % 4 != 0:
        raise GoJSONError("illegal base64 data")
    alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"
    out = bytearray()
    for q in range(0, len(s), 4):
        chunk = s[q:q + 4]
        pad = 0
        if chunk[3] == "=":
            pad = 1
            if chunk[2] == "=":
                pad = 2
            if q + 4 != len(s):
                raise GoJSONError("illegal base64 data")
        vals = []
        for ch in chunk[:4 - pad]:
            k = alpha.find(ch)
            if k < 0:
                raise GoJSONError("illegal base64 data")
            vals.append(k)
        if pad == 2 and "=" in chunk[:2]:
            raise GoJSONError("illegal base64 data")
        n = 0
        for v in vals:
            n = (n << 6) | v
        n <<= 6 * pad
        blk = n.to_bytes(3, "big")
        out += blk[:3 - pad]
    return bytes(out)


def dec_bytes(v):
    """[]byte field: null -> None, string -> base64 decode."""
    if v is None or v[0] == "null":
        return None
    if v[0] != "str":
        raise GoJSONError("cannot unmarshal %s into []byte" % v[0])
    return b64_std_decode(v[1])


def dec_int(v):
    if v is None or v[0] == "null":
        return 0
    if v[0] != "num":
        raise GoJSONError("cannot unmarshal %s into int" % v[0])
    tok = v[1]
    if any(ch in tok for ch in ".eE"):
        raise GoJSONError("cannot unmarshal number %s into int" % tok)
    n = int(tok)
    if not -(1 << 63) <= n < (1 << 63):
        raise GoJSONError("number out of range")
    return n


def dec_string(v):
    if v is None or v[0] == "null":
        return ""
    if v[0] != "str":
        raise GoJSONError("cannot unmarshal %s into string" % v[0])
    return v[1]


def dec_list(v, f):
    """Slice of pointers: null -> None; each element decoded by f (which maps a
    JSON null element to None, i.e. a nil pointer entry)."""
    if v is None or v[0] == "null":
        return None
    if v[0] != "arr":
        raise GoJSONError("cannot unmarshal %s into slice" % v[0])
    return [f(x) for x in v[1]]


def dec_elem(v):
    """mathlib element UnmarshalJSON -> (curve_id, element_bytes) or None for
    JSON null (Go leaves the pointer nil without calling UnmarshalJSON)."""
    if v is None or v[0] == "null":
        return None
    if v[0] != "obj":
        raise GoJSONError("cannot unmarshal %s into curveElement" % v[0])
    curve = dec_int(field(v, "curve"))
    raw = dec_bytes(field(v, "element"))
    return (curve, raw)
