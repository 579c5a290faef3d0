// edn.cpp — Jepsen history.edn -> packed lc_op records (include/lincheck_edn.h).
//
// Host code (no HIP).  Three stages, each on n_threads threads:
//  1. a structural scan finds the top-level forms (strings, character
//     literals, comments and brackets only: no values are built), on pieces
//     cut at newlines and stitched into the serial scan's result;
//  2. the forms are parsed into compact op summaries (type, f, process, index
//     and the parts of :value the register model reads, with EDN-equality
//     identities for keys and values);
//  3. the per-key split (jepsen.independent, register.clj:108), knossos
//     history completion and per-key value interning.
// The rules are those of jepsen/etcd_amd/history.py; tests/test_edn.py holds
// the two to the same records on generated and hand-written histories.
#include "../../../include/lincheck_edn.h"

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

// ------------------------------------------------------------------ scan
bool is_ws(char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == ',' || c == '\f'; }
bool is_delim(char c) {
  return is_ws(c) || c == '(' || c == ')' || c == '[' || c == ']' || c == '{' || c == '}' ||
         c == '"' || c == ';';
}

struct Scanner {
  const char *s;
  size_t n, p = 0;
  const char *err = nullptr;
  size_t err_at = 0;

  bool fail(const char *m) {
    if (!err) err = m, err_at = p;
    return false;
  }
  void ws() {
    for (;;) {
      while (p < n && is_ws(s[p])) p++;
      if (p < n && s[p] == ';') {
        while (p < n && s[p] != '\n') p++;
        continue;
      }
      break;
    }
  }
  bool string() {  // at '"'
    for (p++; p < n; p++) {
      if (s[p] == '\\') {
        p++;
      } else if (s[p] == '"') {
        p++;
        return true;
      }
    }
    return fail("unterminated string");
  }
  void token() {
    while (p < n && !is_delim(s[p])) p++;
  }
  bool coll() {  // at an opening bracket
    int depth = 0;
    while (p < n) {
      const char c = s[p];
      if (c == '"') {
        if (!string()) return false;
        continue;
      }
      if (c == '\\') {  // character literal: \( \" \; ...
        p += 2;
        continue;
      }
      if (c == ';') {
        while (p < n && s[p] != '\n') p++;
        continue;
      }
      if (c == '(' || c == '[' || c == '{') depth++;
      if (c == ')' || c == ']' || c == '}') {
        if (--depth == 0) {
          p++;
          return true;
        }
        if (depth < 0) return fail("unbalanced closing bracket");
      }
      p++;
    }
    return fail("unterminated collection");
  }
  // skip one form (after ws)
  bool form() {
    if (p >= n) return fail("unexpected end of input");
    const char c = s[p];
    if (c == '(' || c == '[' || c == '{') return coll();
    if (c == ')' || c == ']' || c == '}') return fail("unexpected closing bracket");
    if (c == '"') return string();
    if (c == '\\') {
      p += 2;
      token();
      return true;
    }
    if (c == '#') {
      if (p + 1 < n && s[p + 1] == '{') {
        p++;
        return coll();
      }
      if (p + 1 < n && s[p + 1] == '_') {
        p += 2;
        ws();
        if (!form()) return false;
        ws();
        return form();
      }
      if (p + 1 < n && s[p + 1] == '"') {
        p++;
        return string();
      }
      if (p + 1 < n && s[p + 1] == '#') {
        p += 2;
        token();
        return true;
      }
      p++;
      token();  // the tag
      ws();
      return form();
    }
    token();
    return true;
  }
};

using Spans = std::vector<std::pair<size_t, size_t>>;

// Top-level forms of text[p, e) that start before cend, from p (which must be
// a top-level position).  Returns the position after the last form's
// trailing whitespace (>= cend or e), or the error position.
size_t scan_run(const char *text, size_t p, size_t cend, size_t e, Spans &forms,
                const char *&err, size_t &err_at) {
  Scanner sc{text, e, p};
  for (;;) {
    sc.ws();
    if (sc.p >= e || sc.p >= cend) return sc.p;
    const size_t b = sc.p;
    if (!sc.form()) {
      err = sc.err, err_at = sc.err_at;
      return sc.p;
    }
    forms.emplace_back(b, sc.p);
  }
}

// The top-level forms of text[b, e), on up to T threads, equal to one serial
// scan's.  The range is cut after newlines and each piece is scanned as if it
// began at top level (Jepsen writes one op per line, so it nearly always
// does).  A stitch pass walks the pieces in order from the true scan's
// position: a piece whose speculative forms include that position is right
// from there on (the scan is a function of the position alone); one that does
// not (a string or collection spans the cut) is rescanned serially.
bool scan_forms(const char *text, size_t b, size_t e, int T, Spans &forms, const char *&err,
                size_t &err_at) {
  const size_t len = e > b ? e - b : 0;
  const char *mp = getenv("LC_EDN_MIN_PIECE");  // bytes per piece (tests cut small pieces)
  const size_t min_piece = std::max<size_t>(1, mp ? (size_t)atoll(mp) : (size_t)1 << 20);
  T = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(T, 1), len / min_piece));
  if (T == 1) {
    scan_run(text, b, e, e, forms, err, err_at);
    return !err;
  }
  struct Piece {
    size_t beg, end, last = 0, err_at = 0;
    Spans forms;
    const char *err = nullptr;
  };
  std::vector<Piece> pc(T);
  for (int t = 0; t < T; t++) {
    size_t c = b + len * t / T;
    if (t) {
      const void *nl = memchr(text + c, '\n', e - c);
      c = nl ? (size_t)((const char *)nl - text) + 1 : e;
      c = std::max(c, pc[t - 1].beg);
    }
    pc[t].beg = c;
  }
  for (int t = 0; t < T; t++) pc[t].end = t + 1 < T ? pc[t + 1].beg : e;
  {
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++)
      th.emplace_back([&, t] {
        Piece &x = pc[t];
        x.forms.reserve((x.end - x.beg) / 48);
        x.last = scan_run(text, x.beg, x.end, e, x.forms, x.err, x.err_at);
      });
    Piece &x = pc[0];
    x.last = scan_run(text, x.beg, x.end, e, x.forms, x.err, x.err_at);
    for (auto &y : th) y.join();
  }
  size_t total = 0;
  for (auto &x : pc) total += x.forms.size();
  forms.reserve(total);
  size_t pos = b;  // a position of the true scan, at top level
  for (int t = 0; t < T; t++) {
    Piece &x = pc[t];
    if (pos >= x.end) continue;  // a form of an earlier piece covers this one
    Scanner sc{text, e, pos};
    sc.ws();
    pos = sc.p;
    if (pos >= e) break;
    if (pos >= x.end) continue;
    auto it = std::lower_bound(x.forms.begin(), x.forms.end(), std::make_pair(pos, (size_t)0));
    if (it != x.forms.end() && it->first == pos) {  // in step with the true scan
      forms.insert(forms.end(), it, x.forms.end());
      if (x.err) {
        err = x.err, err_at = x.err_at;
        return false;
      }
      pos = x.last;
    } else {
      pos = scan_run(text, pos, x.end, e, forms, err, err_at);
      if (err) return false;
    }
    Spans().swap(x.forms);
  }
  return true;
}

// ----------------------------------------------------------------- parse
enum NT : uint8_t {
  N_NIL, N_BOOL, N_INT, N_BIG, N_FLOAT, N_DEC, N_RATIO, N_STR, N_CHAR, N_KW, N_SYM,
  N_VEC, N_LIST, N_MAP, N_SET, N_TAG
};

struct Node {
  uint8_t t;
  int64_t i;        // N_INT / N_BOOL
  size_t beg, end;  // source span
  uint32_t kid0, nkid;
};

struct Parser {
  const char *s;
  size_t n, p = 0;
  std::vector<Node> nodes;
  std::vector<uint32_t> kids, stack;
  const char *err = nullptr;
  size_t err_at = 0;

  bool fail(const char *m) {
    if (!err) err = m, err_at = p;
    return false;
  }
  uint32_t add(uint8_t t, size_t b, size_t e, int64_t i = 0) {
    nodes.push_back(Node{t, i, b, e, 0, 0});
    return (uint32_t)nodes.size() - 1;
  }
  bool ws() {
    for (;;) {
      while (p < n && is_ws(s[p])) p++;
      if (p < n && s[p] == ';') {
        while (p < n && s[p] != '\n') p++;
        continue;
      }
      if (p + 1 < n && s[p] == '#' && s[p + 1] == '_') {
        p += 2;
        uint32_t drop;
        if (!form(drop)) return false;
        continue;
      }
      return true;
    }
  }
  bool coll(uint8_t t, size_t beg, char close, uint32_t &out) {
    const size_t base = stack.size();
    for (;;) {
      if (!ws()) return false;
      if (p >= n) return fail("unterminated collection");
      if (s[p] == close) {
        p++;
        break;
      }
      if (s[p] == ')' || s[p] == ']' || s[p] == '}') return fail("mismatched closing bracket");
      uint32_t k;
      if (!form(k)) return false;
      stack.push_back(k);
    }
    const uint32_t nk = (uint32_t)(stack.size() - base);
    if (t == N_MAP && (nk & 1)) return fail("map with an odd number of forms");
    out = add(t, beg, p);
    nodes[out].kid0 = (uint32_t)kids.size();
    nodes[out].nkid = nk;
    kids.insert(kids.end(), stack.begin() + base, stack.end());
    stack.resize(base);
    return true;
  }
  bool number(size_t b, size_t e, uint32_t &out) {
    {  // the common case, a plain decimal that fits: what strtoll below would give
      size_t q = b + (s[b] == '+' || s[b] == '-');
      if (e > q && e - q <= 18) {
        int64_t v = 0;
        size_t r = q;
        while (r < e && s[r] >= '0' && s[r] <= '9') v = v * 10 + (s[r++] - '0');
        if (r == e) {
          out = add(N_INT, b, e, s[b] == '-' ? -v : v);
          return true;
        }
      }
    }
    const std::string t(s + b, e - b);
    if (t.find('/') != std::string::npos) {
      out = add(N_RATIO, b, e);
      return true;
    }
    if (t.back() == 'M') {
      out = add(N_DEC, b, e);
      return true;
    }
    if (t.find_first_of(".eE") != std::string::npos && t.compare(0, 2, "0x") && t.compare(0, 3, "-0x")) {
      char *endp;
      strtod(t.c_str(), &endp);
      if (*endp) return fail("malformed number");
      out = add(N_FLOAT, b, e);
      return true;
    }
    std::string d = t;
    if (d.back() == 'N') d.pop_back();
    errno = 0;
    char *endp;
    const long long v = strtoll(d.c_str(), &endp, 10);
    if (*endp) return fail("malformed number");
    if (errno == ERANGE) {
      out = add(N_BIG, b, e);
      return true;
    }
    out = add(N_INT, b, e, (int64_t)v);
    return true;
  }
  bool form(uint32_t &out) {
    if (!ws()) return false;
    if (p >= n) return fail("unexpected end of input");
    const size_t b = p;
    const char c = s[p];
    switch (c) {
      case '(': p++; return coll(N_LIST, b, ')', out);
      case '[': p++; return coll(N_VEC, b, ']', out);
      case '{': p++; return coll(N_MAP, b, '}', out);
      case ')': case ']': case '}': return fail("unexpected closing bracket");
      case '"':
        for (p++; p < n; p++) {
          if (s[p] == '\\') {
            p++;
          } else if (s[p] == '"') {
            p++;
            out = add(N_STR, b, p);
            return true;
          }
        }
        return fail("unterminated string");
      case '\\':
        p += 2;
        while (p < n && !is_delim(s[p])) p++;
        if (p > n) return fail("unterminated character");
        out = add(N_CHAR, b, p);
        return true;
      case '#': {
        if (p + 1 < n && s[p + 1] == '{') {
          p += 2;
          return coll(N_SET, b, '}', out);
        }
        if (p + 1 < n && s[p + 1] == '"') {  // regex: identity by text
          p++;
          uint32_t r;
          if (!form(r)) return false;
          out = add(N_SYM, b, p);
          return true;
        }
        if (p + 1 < n && s[p + 1] == '#') {  // ##Inf ##NaN
          p += 2;
          while (p < n && !is_delim(s[p])) p++;
          out = add(N_SYM, b, p);
          return true;
        }
        p++;
        while (p < n && !is_delim(s[p])) p++;
        if (p == b + 1) return fail("empty tag");
        uint32_t inner;
        if (!form(inner)) return false;
        out = add(N_TAG, b, p);
        nodes[out].kid0 = (uint32_t)kids.size();
        nodes[out].nkid = 1;
        kids.push_back(inner);
        return true;
      }
      default:
        break;
    }
    while (p < n && !is_delim(s[p])) p++;
    const size_t e = p;
    const size_t len = e - b;
    if (c == ':') {
      out = add(N_KW, b, e);
      return true;
    }
    const bool digit = c >= '0' && c <= '9';
    const bool sdigit = (c == '+' || c == '-') && len > 1 && s[b + 1] >= '0' && s[b + 1] <= '9';
    if (digit || sdigit) return number(b, e, out);
    if (len == 3 && !memcmp(s + b, "nil", 3)) {
      out = add(N_NIL, b, e);
      return true;
    }
    if (len == 4 && !memcmp(s + b, "true", 4)) {
      out = add(N_BOOL, b, e, 1);
      return true;
    }
    if (len == 5 && !memcmp(s + b, "false", 5)) {
      out = add(N_BOOL, b, e, 0);
      return true;
    }
    out = add(N_SYM, b, e);
    return true;
  }

  // Identity of a value under EDN / Clojure equality (see header).
  void canon(uint32_t id, std::string &o) const {
    const Node &x = nodes[id];
    switch (x.t) {
      case N_NIL: o += "nil"; return;
      case N_BOOL: o += x.i ? "true" : "false"; return;
      case N_INT: o += std::to_string(x.i); return;
      case N_BIG: {  // beyond int64: normalised digits
        size_t b = x.beg, e = x.end;
        if (s[e - 1] == 'N') e--;
        bool neg = false;
        if (s[b] == '+' || s[b] == '-') neg = s[b++] == '-';
        while (b + 1 < e && s[b] == '0') b++;
        if (neg) o += '-';
        o.append(s + b, e - b);
        return;
      }
      case N_FLOAT: {
        char buf[40];
        snprintf(buf, sizeof buf, "F%.17g", strtod(std::string(s + x.beg, x.end - x.beg).c_str(), nullptr));
        o += buf;
        return;
      }
      case N_DEC: o += 'M'; o.append(s + x.beg, x.end - x.beg); return;
      case N_RATIO: o += 'R'; o.append(s + x.beg, x.end - x.beg); return;
      case N_STR: case N_CHAR: case N_KW: case N_SYM:
        o.append(s + x.beg, x.end - x.beg);
        return;
      case N_VEC: case N_LIST:
        o += '[';
        for (uint32_t k = 0; k < x.nkid; k++) {
          if (k) o += ' ';
          canon(kids[x.kid0 + k], o);
        }
        o += ']';
        return;
      case N_MAP: case N_SET: {
        std::vector<std::string> parts;
        const uint32_t step = x.t == N_MAP ? 2 : 1;
        for (uint32_t k = 0; k < x.nkid; k += step) {
          std::string e;
          canon(kids[x.kid0 + k], e);
          if (step == 2) {
            e += ' ';
            canon(kids[x.kid0 + k + 1], e);
          }
          parts.push_back(std::move(e));
        }
        std::sort(parts.begin(), parts.end());
        o += x.t == N_MAP ? "{" : "#{";
        for (size_t k = 0; k < parts.size(); k++) {
          if (k) o += ", ";
          o += parts[k];
        }
        o += '}';
        return;
      }
      case N_TAG: {
        const Node &in = nodes[kids[x.kid0]];
        size_t e = x.beg + 1;
        while (e < in.beg && !is_delim(s[e])) e++;
        o += '#';
        o.append(s + x.beg + 1, e - x.beg - 1);
        o += ' ';
        canon(kids[x.kid0], o);
        return;
      }
    }
  }
  bool is_pair(uint32_t id) const {
    const Node &x = nodes[id];
    return (x.t == N_VEC || x.t == N_LIST) && x.nkid == 2;
  }
  uint32_t kid(uint32_t id, uint32_t k) const { return kids[nodes[id].kid0 + k]; }
  bool kw_is(uint32_t id, const char *kw) const {
    const Node &x = nodes[id];
    const size_t len = strlen(kw);
    return x.t == N_KW && x.end - x.beg == len && !memcmp(s + x.beg, kw, len);
  }
};

// One value slot of an op: identity (offset/length into the thread's pool)
// and source span (for display).
struct Val {
  uint64_t off = 0;
  uint32_t len = 0;
  uint8_t nil = 1;
  size_t beg = 0, end = 0;
};

// What the checker needs from one op map.
struct POp {
  size_t beg, end;          // the op form
  int64_t process = 0, index = 0;
  int8_t type = -1;         // 0 invoke, 1 ok, 2 fail, 3 info, -1 other
  int8_t f = 3;             // 0 read, 1 write, 2 cas, 3 other
  uint8_t client = 0, has_index = 0, tuple = 0;
  // the (unwrapped) value: [version x], x = [old new] for cas
  uint8_t v_pair = 0, ver_kind = 2, x_pair = 0;  // ver_kind 0 nil, 1 int, 2 other
  int64_t ver = 0;
  Val key, x, x0, x1;
  uint32_t thread = 0;      // owner of the pool
};

struct alignas(128) Chunk {  // one per parse thread: no false sharing of the vector headers
  std::vector<POp> ops;
  std::string pool;
  const char *err = nullptr;
  size_t err_at = 0;
  // the chunk's view of the per-key split: per op, a chunk-local key id
  // (-1 not a client op, -2 a client op without a tuple); per local key, its
  // canonical text and the op where it first appears
  std::vector<int32_t> kid;
  std::vector<std::string_view> lkey;
  std::vector<uint32_t> lfirst;
  bool shared = false;
};

// Local key ids in order of first appearance within the chunk.
void local_keys(Chunk &c, bool independent) {
  c.kid.resize(c.ops.size());
  std::unordered_map<std::string_view, int32_t> ids;
  for (size_t i = 0; i < c.ops.size(); i++) {
    const POp &o = c.ops[i];
    if (!o.client) {
      c.kid[i] = -1;
    } else if (independent && !o.tuple) {
      c.kid[i] = -2;
      c.shared = true;
    } else {  // not independent: every client op is the one key ""
      const std::string_view k = independent ? std::string_view(c.pool.data() + o.key.off, o.key.len)
                                             : std::string_view();
      auto it = ids.find(k);
      if (it == ids.end()) {
        it = ids.emplace(k, (int32_t)c.lkey.size()).first;
        c.lkey.push_back(k);
        c.lfirst.push_back((uint32_t)i);
      }
      c.kid[i] = it->second;
    }
  }
}

void put_val(const Parser &ps, uint32_t id, std::string &pool, Val &v) {
  const Node &x = ps.nodes[id];
  v.beg = x.beg;
  v.end = x.end;
  v.nil = x.t == N_NIL;
  v.off = pool.size();
  ps.canon(id, pool);
  v.len = (uint32_t)(pool.size() - v.off);
}

void parse_chunk(const char *text, const std::vector<std::pair<size_t, size_t>> &forms, size_t f0,
                 size_t f1, bool independent, bool versioned, uint32_t tid, Chunk &out) {
  Parser ps;
  ps.s = text;
  out.ops.reserve(f1 - f0);
  for (size_t fi = f0; fi < f1; fi++) {
    ps.n = forms[fi].second;
    ps.p = forms[fi].first;
    ps.nodes.clear();
    ps.kids.clear();
    uint32_t root;
    if (!ps.form(root)) {
      out.err = ps.err;
      out.err_at = ps.err_at;
      return;
    }
    while (ps.nodes[root].t == N_TAG) root = ps.kid(root, 0);  // #jepsen.history.Op{...}
    POp o;
    o.beg = forms[fi].first;
    o.end = forms[fi].second;
    o.thread = tid;
    if (ps.nodes[root].t != N_MAP) {  // not an op: counted, never checked
      out.ops.push_back(o);
      continue;
    }
    int32_t value = -1;
    const Node &m = ps.nodes[root];
    for (uint32_t k = 0; k < m.nkid; k += 2) {
      const uint32_t key = ps.kids[m.kid0 + k], v = ps.kids[m.kid0 + k + 1];
      const Node &vn = ps.nodes[v];
      if (ps.kw_is(key, ":type")) {
        o.type = ps.kw_is(v, ":invoke") ? 0 : ps.kw_is(v, ":ok") ? 1 : ps.kw_is(v, ":fail") ? 2
                 : ps.kw_is(v, ":info") ? 3 : -1;
      } else if (ps.kw_is(key, ":f")) {
        o.f = ps.kw_is(v, ":read") ? 0 : ps.kw_is(v, ":write") ? 1 : ps.kw_is(v, ":cas") ? 2
              : ps.kw_is(v, ":acquire") ? 4 : ps.kw_is(v, ":release") ? 5 : 3;
      } else if (ps.kw_is(key, ":process")) {
        o.client = vn.t == N_INT;
        o.process = vn.i;
      } else if (ps.kw_is(key, ":index")) {
        if (vn.t == N_INT) o.has_index = 1, o.index = vn.i;
      } else if (ps.kw_is(key, ":value")) {
        value = (int32_t)v;
      }
    }
    if (value >= 0) {
      uint32_t v = (uint32_t)value;
      if (independent && ps.nodes[v].t == N_VEC && ps.nodes[v].nkid == 2) {
        o.tuple = 1;
        put_val(ps, ps.kid(v, 0), out.pool, o.key);
        v = ps.kid(v, 1);
      }
      if (!versioned) {  // knossos (cas-)register: the value is x itself
        o.v_pair = 1;
        o.ver_kind = 0;
        put_val(ps, v, out.pool, o.x);
        if (ps.is_pair(v)) {
          o.x_pair = 1;
          put_val(ps, ps.kid(v, 0), out.pool, o.x0);
          put_val(ps, ps.kid(v, 1), out.pool, o.x1);
        }
      } else if (ps.is_pair(v)) {
        o.v_pair = 1;
        const Node &ver = ps.nodes[ps.kid(v, 0)];
        o.ver_kind = ver.t == N_NIL ? 0 : ver.t == N_INT ? 1 : 2;
        o.ver = ver.i;
        const uint32_t x = ps.kid(v, 1);
        put_val(ps, x, out.pool, o.x);
        if (ps.is_pair(x)) {
          o.x_pair = 1;
          put_val(ps, ps.kid(x, 0), out.pool, o.x0);
          put_val(ps, ps.kid(x, 1), out.pool, o.x1);
        }
      }
    }
    out.ops.push_back(o);
  }
}

}  // namespace

struct lc_edn_history {
  const char *text = nullptr;
  int64_t n_events = 0;
  std::vector<lc_op> ops;
  std::vector<int64_t> key_off;
  // lc_op32 records (ABI 4) and key bases, made on first request
  std::vector<lc_op32> ops32;
  std::vector<int64_t> key_base;
  bool packed32 = false;
  // lc_op16 records (round 6), made on first request: 1 packed, -1 an id
  // does not fit 15 bits
  std::vector<lc_op16> ops16;
  int packed16 = 0;
  std::vector<std::string> keys;                  // display text
  std::vector<std::vector<std::string>> values;   // per key: display text by id
  std::vector<std::pair<size_t, size_t>> inv, comp;  // per record: op spans (comp beg == end: none)
  std::string last;
};

namespace {

struct Interner {
  std::unordered_map<std::string_view, int32_t> ids;  // views into the chunks' pools
  std::vector<std::string> *shown;
  const char *text;
  int64_t operator()(const std::vector<Chunk> &ch, const POp &o, const Val &v) {
    if (v.nil) return LC_NIL;
    const std::string_view k(ch[o.thread].pool.data() + v.off, v.len);
    auto it = ids.find(k);
    if (it != ids.end()) return it->second;
    const int32_t id = (int32_t)shown->size();
    ids.emplace(k, id);
    shown->emplace_back(text + v.beg, v.end - v.beg);
    return id;
  }
};

}  // namespace

extern "C" {

int lc_edn_parse(const char *text, size_t len, int64_t flags, int n_threads,
                 lc_edn_history **out, char *err, size_t errlen) {
  auto fail = [&](const char *m, size_t at) {
    if (err && errlen) snprintf(err, errlen, "EDN: %s at byte %zu", m, at);
    return -EINVAL;
  };
  if (!out || (!text && len)) return fail("null argument", 0);
  *out = nullptr;
  const bool independent = flags & LC_EDN_INDEPENDENT;
  const int64_t model = flags & LC_EDN_MODEL_MASK;
  if (model > LC_EDN_MUTEX) return fail("unknown model in flags", 0);
  const bool timing = getenv("LC_EDN_TIMING") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto lap = [&](const char *what) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "lc_edn %-10s %8.1f ms\n", what,
            std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  // 1. top-level forms (inside a single wrapping vector, if that is the file)
  const int T0 = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  Scanner sc{text, len};
  sc.ws();
  size_t stop = len;
  Spans forms;
  const char *serr = nullptr;
  size_t serr_at = 0;
  bool scanned = false;
  if (sc.p < len && text[sc.p] == '[') {
    size_t last = len;
    while (last > sc.p && is_ws(text[last - 1])) last--;
    // the common wrapped file, "[op op ...]": scan the inside directly
    if (last > sc.p + 1 && text[last - 1] == ']' &&
        scan_forms(text, sc.p + 1, last - 1, T0, forms, serr, serr_at) &&
        (forms.empty() || forms.back().second <= last - 1)) {
      scanned = true;
    } else {
      forms.clear();
      serr = nullptr;
      Scanner probe{text, len, sc.p};
      if (!probe.form()) return fail(probe.err, probe.err_at);
      probe.ws();
      if (probe.p == len) {  // one vector holding the ops
        sc.p++;
        stop = probe.p - 1;
        while (stop > sc.p && text[stop] != ']') stop--;
      }
    }
  }
  if (!scanned && !scan_forms(text, sc.p, stop, T0, forms, serr, serr_at))
    return fail(serr, serr_at);
  lap("scan");
  // 2. parse forms in parallel
  int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)T0, forms.size() / 4096 + 1));
  std::vector<Chunk> ch(T);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) {
      const size_t f0 = forms.size() * t / T, f1 = forms.size() * (t + 1) / T;
      th.emplace_back([&, f0, f1, t] {
        const auto a = std::chrono::steady_clock::now();
        parse_chunk(text, forms, f0, f1, independent, model == LC_EDN_VERSIONED_REGISTER,
                    (uint32_t)t, ch[t]);
        if (!ch[t].err) local_keys(ch[t], independent);
        if (timing)
          fprintf(stderr, "  thread %d: %zu forms %.1f ms\n", t, f1 - f0,
                  std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count());
      });
    }
    for (auto &x : th) x.join();
  }
  if (timing) fprintf(stderr, "lc_edn parse threads %d over %zu forms\n", T, forms.size());
  for (auto &c : ch)
    if (c.err) return fail(c.err, c.err_at);
  lap("parse");
  // 3. keys in order of first appearance (client ops with a tuple value): the
  // chunks' local keys are merged in chunk order, then every chunk scatters
  // its ops into flat per-key lists, file order within a key
  auto par = [](int n, auto fn) {
    std::vector<std::thread> th;
    for (int t = 1; t < n; t++) th.emplace_back(fn, t);
    fn(0);
    for (auto &x : th) x.join();
  };
  auto *h = new lc_edn_history();
  h->text = text;
  h->n_events = (int64_t)forms.size();
  std::vector<int64_t> first_pos(T + 1, 0);
  for (int t = 0; t < T; t++) first_pos[t + 1] = first_pos[t] + (int64_t)ch[t].ops.size();
  std::vector<std::vector<int32_t>> gid(T);  // per chunk: local key -> key
  bool any_shared = false;
  {
    std::unordered_map<std::string_view, int32_t> key_ids;
    if (!independent) {
      key_ids.emplace(std::string_view(), 0);
      h->keys.push_back("nil");
    }
    for (int t = 0; t < T; t++) {
      any_shared |= ch[t].shared;
      gid[t].resize(ch[t].lkey.size());
      for (size_t l = 0; l < ch[t].lkey.size(); l++) {
        auto it = key_ids.find(ch[t].lkey[l]);
        if (it == key_ids.end()) {
          it = key_ids.emplace(ch[t].lkey[l], (int32_t)h->keys.size()).first;
          const POp &o = ch[t].ops[ch[t].lfirst[l]];
          h->keys.emplace_back(text + o.key.beg, o.key.end - o.key.beg);
        }
        gid[t][l] = it->second;
      }
    }
  }
  const size_t K = h->keys.size();
  std::vector<int64_t> sub_off(K + 1, 0);
  std::vector<std::pair<int32_t, int32_t>> sub;  // (chunk, op), key-major
  if (!any_shared) {
    std::vector<int64_t> at((size_t)T * K, 0);  // per chunk and key: count, then write position
    par(T, [&](int t) {
      int64_t *c = at.data() + (size_t)t * K;
      for (const int32_t l : ch[t].kid)
        if (l >= 0) c[gid[t][l]]++;
    });
    int64_t run = 0;
    for (size_t k = 0; k < K; k++) {
      sub_off[k] = run;
      for (int t = 0; t < T; t++) {
        const int64_t c = at[(size_t)t * K + k];
        at[(size_t)t * K + k] = run;
        run += c;
      }
    }
    sub_off[K] = run;
    sub.resize((size_t)run);
    par(T, [&](int t) {
      int64_t *w = at.data() + (size_t)t * K;
      const auto &kid = ch[t].kid;
      for (size_t i = 0; i < kid.size(); i++)
        if (kid[i] >= 0) sub[(size_t)w[gid[t][kid[i]]]++] = {t, (int32_t)i};
    });
  } else {  // rare: non-tuple client ops go to every key, in file order
    std::vector<std::vector<std::pair<int32_t, int32_t>>> lists(K);
    for (int t = 0; t < T; t++) {
      for (size_t i = 0; i < ch[t].kid.size(); i++) {
        const int32_t l = ch[t].kid[i];
        if (l >= 0) {
          lists[gid[t][l]].emplace_back(t, (int32_t)i);
        } else if (l == -2) {
          for (auto &s : lists) s.emplace_back(t, (int32_t)i);
        }
      }
    }
    for (size_t k = 0; k < K; k++) {
      sub_off[k + 1] = sub_off[k] + (int64_t)lists[k].size();
      sub.insert(sub.end(), lists[k].begin(), lists[k].end());
    }
  }
  lap("split");
  // 4. per key: completion + packing, keys in parallel
  struct KeyOut {
    std::vector<lc_op> recs;
    std::vector<std::pair<size_t, size_t>> inv, comp;
    std::vector<std::string> values;
  };
  std::vector<KeyOut> ko(K);
  auto do_keys = [&](size_t k0, size_t k1) {
    for (size_t k = k0; k < k1; k++) {
      struct R {
        int32_t ic, ii, cc = -1, ci = -1;  // invoke / completion (chunk, op)
        int64_t call, ret;
        int8_t type;  // 1 ok, 2 fail, 3 info
      };
      std::vector<R> rs;
      std::unordered_map<int64_t, int32_t> pending;
      for (int64_t j = sub_off[k]; j < sub_off[k + 1]; j++) {
        const auto &e = sub[(size_t)j];
        const POp &o = ch[e.first].ops[e.second];
        const int64_t idx = o.has_index ? o.index : first_pos[e.first] + e.second;
        if (o.type == 0) {
          R r;
          r.ic = e.first;
          r.ii = e.second;
          r.call = idx;
          r.ret = LC_INF;
          r.type = 3;
          pending[o.process] = (int32_t)rs.size();
          rs.push_back(r);
        } else if (o.type > 0) {
          auto it = pending.find(o.process);
          if (it == pending.end()) continue;  // completion without invoke: ignored
          R &r = rs[it->second];
          pending.erase(it);
          r.cc = e.first;
          r.ci = e.second;
          r.type = o.type;
          if (o.type == 1) r.ret = idx;
        }
      }
      KeyOut &out = ko[k];
      if (model == LC_EDN_MUTEX) out.values = {"free", "held"};
      Interner in;
      in.shown = &out.values;
      in.text = text;
      for (const R &r : rs) {
        if (r.type == 2) continue;  // :fail pairs are dropped
        const POp &inv = ch[r.ic].ops[r.ii];
        const POp &vo = r.type == 1 ? ch[r.cc].ops[r.ci] : inv;  // :ok copies its value in
        lc_op rec{inv.f, LC_NIL, LC_NIL, LC_NIL, r.call, r.ret};
        const bool shape = vo.v_pair && vo.ver_kind != 2 && (inv.f != LC_F_CAS || vo.x_pair);
        if (model == LC_EDN_MUTEX) {  // acquire: CAS free(0) -> held(1); release: the reverse
          rec.f = inv.f == 4 || inv.f == 5 ? LC_F_CAS : 3;
          if (rec.f == LC_F_CAS) rec.value = inv.f == 4 ? 1 : 0, rec.expected = inv.f == 4 ? 0 : 1;
        } else if (inv.f > LC_F_CAS || !shape || (model == LC_EDN_REGISTER && inv.f == LC_F_CAS)) {
          rec.f = 3;
        } else {
          rec.version = vo.ver_kind == 0 ? LC_NIL : vo.ver;
          if (inv.f == LC_F_CAS) {
            rec.value = in(ch, vo, vo.x1);  // history.py interns new before old
            rec.expected = in(ch, vo, vo.x0);
          } else {
            rec.value = in(ch, vo, vo.x);
          }
        }
        out.recs.push_back(rec);
        out.inv.emplace_back(inv.beg, inv.end);
        if (r.cc >= 0) {
          const POp &c = ch[r.cc].ops[r.ci];
          out.comp.emplace_back(c.beg, c.end);
        } else {
          out.comp.emplace_back(0, 0);
        }
      }
    }
  };
  const int KT = (int)std::max<size_t>(1, std::min<size_t>((size_t)T, K / 64 + 1));
  par(KT, [&](int t) { do_keys(K * t / KT, K * (t + 1) / KT); });
  lap("complete");
  h->key_off.assign(K + 1, 0);
  for (size_t k = 0; k < K; k++) h->key_off[k + 1] = h->key_off[k] + (int64_t)ko[k].recs.size();
  h->ops.resize((size_t)h->key_off[K]);
  h->inv.resize((size_t)h->key_off[K]);
  h->comp.resize((size_t)h->key_off[K]);
  h->values.resize(K);
  par(KT, [&](int t) {
    for (size_t k = K * t / KT; k < K * (t + 1) / KT; k++) {
      const size_t o = (size_t)h->key_off[k];
      std::copy(ko[k].recs.begin(), ko[k].recs.end(), h->ops.begin() + o);
      std::copy(ko[k].inv.begin(), ko[k].inv.end(), h->inv.begin() + o);
      std::copy(ko[k].comp.begin(), ko[k].comp.end(), h->comp.begin() + o);
      h->values[k] = std::move(ko[k].values);
      ko[k] = KeyOut();
    }
  });
  lap("gather");
  *out = h;
  return 0;
}

int64_t lc_edn_n_keys(const lc_edn_history *h) { return h ? (int64_t)h->keys.size() : 0; }
int64_t lc_edn_n_ops(const lc_edn_history *h) { return h ? (int64_t)h->ops.size() : 0; }
int64_t lc_edn_n_events(const lc_edn_history *h) { return h ? h->n_events : 0; }
const lc_op *lc_edn_ops(const lc_edn_history *h) { return h ? h->ops.data() : nullptr; }
const int64_t *lc_edn_key_off(const lc_edn_history *h) { return h ? h->key_off.data() : nullptr; }

// The 24-byte form lc_check32 takes (include/lincheck.h, ABI 4), narrowed by
// lc_pack32's rules once, on first request.
static int pack32(lc_edn_history *h) {
  if (h->packed32) return 0;
  const int64_t nk = (int64_t)h->key_off.size() - 1;
  h->ops32.resize(std::max<size_t>(1, h->ops.size()));
  h->key_base.resize(std::max<int64_t>(1, nk));
  if (int rc = lc_pack32(h->ops.data(), h->key_off.data(), nk, h->ops32.data(), h->key_base.data()))
    return rc;
  h->packed32 = true;
  return 0;
}
const lc_op32 *lc_edn_ops32(lc_edn_history *h) { return h && !pack32(h) ? h->ops32.data() : nullptr; }
const int64_t *lc_edn_key_base(lc_edn_history *h) {
  return h && !pack32(h) ? h->key_base.data() : nullptr;
}

// The 16-byte form lc_check16 takes, by lc_pack16's rules (its key bases are
// lc_pack32's: lc_edn_key_base), or null when an id does not fit 15 bits.
const lc_op16 *lc_edn_ops16(lc_edn_history *h) {
  if (!h) return nullptr;
  if (h->packed16 == 0) {
    const int64_t nk = (int64_t)h->key_off.size() - 1;
    h->ops16.resize(std::max<size_t>(1, h->ops.size()));
    std::vector<int64_t> base((size_t)std::max<int64_t>(1, nk));
    h->packed16 = lc_pack16(h->ops.data(), h->key_off.data(), nk, h->ops16.data(), base.data()) ? -1 : 1;
  }
  return h->packed16 > 0 ? h->ops16.data() : nullptr;
}

const char *lc_edn_key(const lc_edn_history *h, int64_t key) {
  if (!h || key < 0 || key >= (int64_t)h->keys.size()) return nullptr;
  return h->keys[key].c_str();
}

const char *lc_edn_op_text(const lc_edn_history *h, int64_t rec, int which) {
  if (!h || rec < 0 || rec >= (int64_t)h->ops.size() || which < 0 || which > 1) return nullptr;
  const auto &sp = which ? h->comp[rec] : h->inv[rec];
  if (sp.second <= sp.first) return nullptr;
  auto *mh = const_cast<lc_edn_history *>(h);
  mh->last.assign(h->text + sp.first, sp.second - sp.first);
  return mh->last.c_str();
}

const char *lc_edn_value(const lc_edn_history *h, int64_t key, int64_t id) {
  if (!h || key < 0 || key >= (int64_t)h->values.size()) return nullptr;
  if (id < 0 || id >= (int64_t)h->values[key].size()) return nullptr;
  return h->values[key][id].c_str();
}

void lc_edn_free(lc_edn_history *h) { delete h; }

}  // extern "C"
