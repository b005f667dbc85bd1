"""Go ``encoding/json`` restated for the zkatdlog wire format (TEST INFRASTRUCTURE ONLY).

Encoding follows ``json.Marshal``: struct fields in declaration order, no
whitespace, ``[]byte`` as standard base64 with padding, nil slices/pointers as
``null``, HTML-safe string escaping.  mathlib's G1/G2/Zr elements marshal as
``{"curve":<CurveID>,"element":<base64(Bytes())>}`` ([EXT]).

Decoding follows ``json.Unmarshal``: object keys match struct fields exactly
or case-insensitively, unknown keys are ignored, a later duplicate overwrites
an earlier one, ``null`` leaves a nil pointer/slice, ``[]byte`` is decoded by
``base64.StdEncoding`` (``\\r``/``\\n`` ignored, padding required).
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
class _Parser:
    """Minimal RFC 8259 parser that keeps object members as an ordered list of
    (key, value) pairs, so duplicate keys survive to the typed decoder."""

    def __init__(self, text):
        if isinstance(text, (bytes, bytearray)):
            try:
                text = bytes(text).decode("utf-8")
            except UnicodeDecodeError as e:
                raise GoJSONError("invalid utf-8") from e
        self.s = text
        self.i = 0

    def ws(self):
        s, i = self.s, self.i
        while i < len(s) and s[i] in " \t\r\n":
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
        if c == "{":
            return self.obj()
        if c == "[":
            return self.arr()
        if c == '"':
            return ("str", self.string())
        if self.s.startswith("null", self.i):
            self.i += 4
            return ("null", None)
        if self.s.startswith("true", self.i):
            self.i += 4
            return ("bool", True)
        if self.s.startswith("false", self.i):
            self.i += 5
            return ("bool", False)
        return self.number()

    def obj(self):
        self.i += 1
        pairs = []
        self.ws()
        if self.i < len(self.s) and self.s[self.i] == "}":
            self.i += 1
            return ("obj", pairs)
        while True:
            self.ws()
            if self.i >= len(self.s) or self.s[self.i] != '"':
                raise GoJSONError("expected object key")
            k = self.string()
            self.ws()
            if self.i >= len(self.s) or self.s[self.i] != ":":
                raise GoJSONError("expected ':'")
            self.i += 1
            v = self.value()
            pairs.append((k, v))
            self.ws()
            if self.i >= len(self.s):
                raise GoJSONError("unexpected end")
            if self.s[self.i] == ",":
                self.i += 1
                continue
            if self.s[self.i] == "}":
                self.i += 1
                return ("obj", pairs)
            raise GoJSONError("expected ',' or '}'")

    def arr(self):
        self.i += 1
        items = []
        self.ws()
        if self.i < len(self.s) and self.s[self.i] == "]":
            self.i += 1
            return ("arr", items)
        while True:
            items.append(self.value())
            self.ws()
            if self.i >= len(self.s):
                raise GoJSONError("unexpected end")
            if self.s[self.i] == ",":
                self.i += 1
                continue
            if self.s[self.i] == "]":
                self.i += 1
                return ("arr", items)
            raise GoJSONError("expected ',' or ']'")

    def string(self):
        s = self.s
        i = self.i + 1
        out = []
        while True:
            if i >= len(s):
                raise GoJSONError("unterminated string")
            c = s[i]
            if c == '"':
                self.i = i + 1
                return "".join(out)
            if c == "\\":
                i += 1
                if i >= len(s):
                    raise GoJSONError("bad escape")
                e = s[i]
                m = {'"': '"', "\\": "\\", "/": "/", "b": "\b", "f": "\f",
                     "n": "\n", "r": "\r", "t": "\t"}
                if e in m:
                    out.append(m[e])
                    i += 1
                elif e == "u":
                    h = s[i + 1:i + 5]
                    if len(h) != 4 or any(ch not in "0123456789abcdefABCDEF" for ch in h):
                        raise GoJSONError("bad \\u escape")
                    cp = int(h, 16)
                    i += 5
                    if 0xD800 <= cp < 0xDC00 and s[i:i + 2] == "\\u":
                        h2 = s[i + 2:i + 6]
                        try:
                            lo = int(h2, 16)
                        except ValueError:
                            lo = -1
                        if 0xDC00 <= lo < 0xE000:
                            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00)
                            i += 6
                        else:
                            cp = 0xFFFD
                    elif 0xD800 <= cp < 0xE000:
                        cp = 0xFFFD
                    out.append(chr(cp))
                else:
                    raise GoJSONError("bad escape")
                continue
            if ord(c) < 0x20:
                raise GoJSONError("control character in string")
            out.append(c)
            i += 1

    def number(self):
        s = self.s
        j = self.i
        if j < len(s) and s[j] == "-":
            j += 1
        if j < len(s) and s[j] == "0":
            j += 1
        elif j < len(s) and s[j].isdigit():
            while j < len(s) and s[j].isdigit():
                j += 1
        else:
            raise GoJSONError("invalid character")
        if j < len(s) and s[j] == ".":
            j += 1
            if not (j < len(s) and s[j].isdigit()):
                raise GoJSONError("bad number")
            while j < len(s) and s[j].isdigit():
                j += 1
        if j < len(s) and s[j] in "eE":
            j += 1
            if j < len(s) and s[j] in "+-":
                j += 1
            if not (j < len(s) and s[j].isdigit()):
                raise GoJSONError("bad number")
            while j < len(s) and s[j].isdigit():
                j += 1
        tok = s[self.i:j]
        self.i = j
        return ("num", tok)


def parse(text):
    return _Parser(text).parse()


def field(obj, name):
    """Go struct-field lookup: the LAST member whose key equals ``name`` exactly
    or case-insensitively (Go applies members in order, so the last wins).
    Returns None when the key is absent (zero value)."""
    if obj[0] != "obj":
        raise GoJSONError("cannot unmarshal %s into struct" % obj[0])
    found = None
    lname = name.lower()
    for k, v in obj[1]:
        if k == name or k.lower() == lname:
            found = v
    return found


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
