// Native host featurizer + JSONL pair-dataset reader (C ABI, loaded with ctypes).
//
// Implements the tokenizer rules of the reference utils/data_utils.py
// (clean_str :11-19, get_text_feature_splits :21-55, pad_sentences :57-68,
// build_input_data :83-92) and the record schema consumed by
// dssm_cnn_v2/data_helpers.py:128-197 ({'q','doc_corr','doc_incorr'[J]}).
// The Python restatement lives in dnn_page_vectors_amd/data/text.py; tests
// check the two agree (golden cases + hypothesis fuzzing).
//
// Design: text is decoded to code points once, cleaned + lower-cased in place,
// re-encoded to UTF-8 with a code-point -> byte offset table so every token is
// a byte range (no per-token allocation). Ids come from a hash map (exact vocab)
// or FNV-1a word hashing (id = 1 + h % (V-1), 0 = PAD). Batches are split over
// a std::thread pool; ctypes drops the GIL for the whole call.
#include <atomic>
#include <clocale>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cwctype>
#include <fcntl.h>
#include <locale.h>
#include <mutex>
#include <string>
#include <string_view>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <vector>

namespace {

locale_t utf8_locale() {
  static locale_t loc = [] {
    locale_t l = newlocale(LC_CTYPE_MASK, "C.UTF-8", (locale_t)0);
    if (!l) l = newlocale(LC_CTYPE_MASK, "en_US.UTF-8", (locale_t)0);
    return l;
  }();
  return loc;
}

inline bool is_word_cp(uint32_t c) {
  if (c < 128) return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_';
  locale_t l = utf8_locale();
  return l ? iswalnum_l((wint_t)c, l) != 0 : false;
}

inline bool keep_cp(uint32_t c) {
  // [\wäöüß€#\n.$]
  switch (c) {
    case 0xE4: case 0xF6: case 0xFC: case 0xDF: case 0x20AC:
    case '#': case '\n': case '.': case '$':
      return true;
    default:
      return is_word_cp(c);
  }
}

inline uint32_t lower_cp(uint32_t c) {
  if (c < 128) return (c >= 'A' && c <= 'Z') ? c + 32 : c;
  locale_t l = utf8_locale();
  return l ? (uint32_t)towlower_l((wint_t)c, l) : c;
}

// Decode UTF-8 (invalid bytes -> U+FFFD, like errors="replace").
void decode_utf8(const char* s, size_t n, std::vector<uint32_t>& out) {
  out.clear();
  out.reserve(n);
  size_t i = 0;
  const unsigned char* u = (const unsigned char*)s;
  while (i < n) {
    unsigned char c = u[i];
    uint32_t cp;
    int len;
    if (c < 0x80) { cp = c; len = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; len = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; len = 3; }
    else if ((c >> 3) == 30) { cp = c & 0x07; len = 4; }
    else { out.push_back(0xFFFD); ++i; continue; }
    if (i + len > n) { out.push_back(0xFFFD); ++i; continue; }
    bool ok = true;
    for (int k = 1; k < len; ++k) {
      if ((u[i + k] >> 6) != 2) { ok = false; break; }
      cp = (cp << 6) | (u[i + k] & 0x3F);
    }
    if (!ok) { out.push_back(0xFFFD); ++i; continue; }
    out.push_back(cp);
    i += len;
  }
}

inline void encode_cp(uint32_t cp, std::string& o) {
  if (cp < 0x80) o.push_back((char)cp);
  else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
  else if (cp < 0x10000) {
    o.push_back((char)(0xE0 | (cp >> 12))); o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    o.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    o.push_back((char)(0xF0 | (cp >> 18))); o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    o.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); o.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

// ------------------------------------------------------- HTML normaliser --
// utils/word2vec_normalizer.py:116-146 (Word2VecTextNormalizer.preprocess_line) as restated
// in data/text.py::normalize_html_line: strip, drop ';lt;'-style fragments, html.unescape,
// strip tags (HTMLParser data only, charrefs converted again), drop \n \r \t, collapse dot
// runs and pad them with spaces, per-word [^\wäöüß€\n.$] -> ' ' + lower-case, collapse
// whitespace runs.  Entity names come from Python's own table (html_entities.inc).
struct HtmlEntity { const char* name; const char* utf8; };
struct NumericFix { uint32_t cp; const char* utf8; };
#include "html_entities.inc"

using U32 = std::u32string;

inline bool py_space(uint32_t c) {  // str.isspace / re \s for str patterns
  return (c >= 9 && c <= 13) || (c >= 0x1C && c <= 0x20) || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

void append_utf8(const char* s, U32& o) {
  std::vector<uint32_t> cps;
  decode_utf8(s, strlen(s), cps);
  o.append(cps.begin(), cps.end());
}

const HtmlEntity* find_entity(const std::string& name) {
  size_t lo = 0, hi = sizeof(kHtmlEntities) / sizeof(kHtmlEntities[0]);
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    int c = strcmp(kHtmlEntities[mid].name, name.c_str());
    if (c == 0) return &kHtmlEntities[mid];
    if (c < 0) lo = mid + 1; else hi = mid;
  }
  return nullptr;
}

std::string to_utf8(const U32& s, size_t b, size_t e) {
  std::string o;
  for (size_t i = b; i < e; ++i) encode_cp(s[i], o);
  return o;
}

// html.unescape: &(#[0-9]+;?|#[xX][0-9a-fA-F]+;?|[^\t\n\f <&#;]{1,32};?)
U32 html_unescape(const U32& s) {
  if (s.find(U'&') == U32::npos) return s;
  U32 o;
  o.reserve(s.size());
  const size_t n = s.size();
  size_t i = 0;
  while (i < n) {
    if (s[i] != U'&') { o.push_back(s[i++]); continue; }
    size_t j = i + 1;
    if (j < n && s[j] == U'#') {
      bool hex = j + 1 < n && (s[j + 1] == U'x' || s[j + 1] == U'X');
      size_t d = j + (hex ? 2 : 1), k = d;
      uint64_t num = 0;
      auto digit = [&](uint32_t c, int& v) {
        if (c >= '0' && c <= '9') { v = (int)(c - '0'); return true; }
        if (hex && c >= 'a' && c <= 'f') { v = (int)(c - 'a' + 10); return true; }
        if (hex && c >= 'A' && c <= 'F') { v = (int)(c - 'A' + 10); return true; }
        return false;
      };
      int v;
      while (k < n && digit(s[k], v)) {
        num = num * (hex ? 16 : 10) + (uint64_t)v;
        if (num > 0x110000) num = 0x110000;  // anything past 0x10FFFF is U+FFFD
        ++k;
      }
      if (k == d) { o.push_back(s[i++]); continue; }  // "&#" without digits: literal
      if (k < n && s[k] == U';') ++k;
      bool done = false;
      for (const auto& f : kInvalidCharrefs)
        if (f.cp == num) { append_utf8(f.utf8, o); done = true; break; }
      if (!done) {
        if ((num >= 0xD800 && num <= 0xDFFF) || num > 0x10FFFF) o.push_back(0xFFFD);
        else {
          bool invalid = false;
          for (uint32_t c : kInvalidCodepoints) if (c == num) { invalid = true; break; }
          if (!invalid) o.push_back((uint32_t)num);
        }
      }
      i = k;
      continue;
    }
    size_t k = j;
    while (k < n && k - j < 32) {
      uint32_t c = s[k];
      if (c == U'\t' || c == U'\n' || c == U'\f' || c == U' ' || c == U'<' || c == U'&' || c == U'#' || c == U';')
        break;
      ++k;
    }
    if (k == j) { o.push_back(s[i++]); continue; }
    if (k < n && s[k] == U';') ++k;
    std::string name = to_utf8(s, j, k);
    if (const HtmlEntity* e = find_entity(name)) {
      append_utf8(e->utf8, o);
    } else {
      bool hit = false;
      for (size_t x = k - j - 1; x >= 2; --x) {  // longest known prefix (legacy names without ';')
        if (const HtmlEntity* e2 = find_entity(to_utf8(s, j, j + x))) {
          append_utf8(e2->utf8, o);
          o.append(s, j + x, k - (j + x));
          hit = true;
          break;
        }
      }
      if (!hit) { o.push_back(U'&'); o.append(s, j, k - j); }
    }
    i = k;
  }
  return o;
}

inline bool ascii_alpha(uint32_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
inline uint32_t ascii_lower(uint32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

bool ieq_at(const U32& s, size_t i, const char* lit) {  // ASCII case-insensitive prefix match
  for (size_t k = 0; lit[k]; ++k)
    if (i + k >= s.size() || ascii_lower(s[i + k]) != (uint32_t)lit[k]) return false;
  return true;
}

// html.parser.HTMLParser(convert_charrefs=True) fed one line and closed: the concatenation of
// its handle_data() calls.  Start / end tags, comments, declarations and processing
// instructions produce no data; script / style content is raw data (no unescape); an
// unterminated construct at the end of the line swallows the rest, as the parser's close() does.
U32 html_strip_tags(const U32& s) {
  U32 o;
  const size_t n = s.size();
  size_t i = 0;
  std::string cdata;  // "script" / "style" while inside one
  while (i < n) {
    if (!cdata.empty()) {  // raw text up to </cdata\s*>
      size_t k = i;
      for (; k < n; ++k) {
        if (s[k] != U'<' || k + 1 >= n || s[k + 1] != U'/') continue;
        size_t m = k + 2;
        while (m < n && py_space(s[m])) ++m;
        if (!ieq_at(s, m, cdata.c_str())) continue;
        m += cdata.size();
        while (m < n && py_space(s[m])) ++m;
        if (m < n && s[m] == U'>') { o.append(s, i, k - i); i = m + 1; cdata.clear(); break; }
      }
      if (k >= n) return o;  // unterminated script/style: dropped
      continue;
    }
    size_t j = s.find(U'<', i);
    if (j == U32::npos) j = n;
    if (j > i) o += html_unescape(s.substr(i, j - i));
    i = j;
    if (i >= n) break;
    if (i + 1 < n && ascii_alpha(s[i + 1])) {  // start tag: name, attributes (quoted values may hold '>')
      size_t k = i + 1, nb = k;
      while (k < n && s[k] != U'\t' && s[k] != U'\n' && s[k] != U'\r' && s[k] != U'\f' && s[k] != U' ' &&
             s[k] != U'/' && s[k] != U'>' && s[k] != 0)
        ++k;
      std::string name;
      for (size_t t = nb; t < k; ++t) name.push_back((char)ascii_lower(s[t] < 128 ? s[t] : '?'));
      uint32_t q = 0;
      for (; k < n; ++k) {
        if (q) { if (s[k] == q) q = 0; continue; }
        if (s[k] == U'"' || s[k] == U'\'') {
          if (k > 0 && (s[k - 1] == U'=' || py_space(s[k - 1]))) q = s[k];
          continue;
        }
        if (s[k] == U'>') break;
      }
      if (k >= n) return o;  // unterminated start tag: the rest is dropped
      bool selfclose = k > 0 && s[k - 1] == U'/';
      if (!selfclose && (name == "script" || name == "style")) cdata = name;
      i = k + 1;
    } else if (i + 1 < n && s[i + 1] == U'/') {
      size_t k = s.find(U'>', i + 1);
      if (k == U32::npos) {
        if (i + 2 == n) o += U"</";
        return o;
      }
      i = k + 1;
    } else if (ieq_at(s, i, "<!--")) {
      size_t k = i + 4;
      for (; k < n; ++k) {  // --\s*>
        if (s[k] != U'-' || k + 1 >= n || s[k + 1] != U'-') continue;
        size_t m = k + 2;
        while (m < n && py_space(s[m])) ++m;
        if (m < n && s[m] == U'>') { k = m; break; }
      }
      if (k >= n) return o;
      i = k + 1;
    } else if (i + 1 < n && (s[i + 1] == U'!' || s[i + 1] == U'?')) {
      size_t k = s.find(U'>', i + 2);
      if (k == U32::npos) return o;
      i = k + 1;
    } else {
      o.push_back(U'<');
      ++i;
    }
  }
  return o;
}

inline bool w2v_keep(uint32_t c) {  // [\wäöüß€\n.$]
  switch (c) {
    case 0xE4: case 0xF6: case 0xFC: case 0xDF: case 0x20AC: case '\n': case '.': case '$':
      return true;
    default:
      return is_word_cp(c);
  }
}

// normalize_html_line on code points (in place in `cps`)
void html_normalize(std::vector<uint32_t>& cps) {
  size_t b = 0, e = cps.size();
  while (b < e && py_space(cps[b])) ++b;
  while (e > b && py_space(cps[e - 1])) --e;
  if (b == e) return;  // blank line: returned unchanged
  U32 s(cps.begin() + b, cps.begin() + e);
  for (const char32_t* frag : {U";lt;", U";gt;", U";amp;", U";apos;", U";quot;"}) {
    const U32 f(frag);
    for (size_t p = s.find(f); p != U32::npos; p = s.find(f, p)) s.erase(p, f.size());
  }
  s = html_strip_tags(html_unescape(s));
  U32 t;  // drop \n \r \t; dot runs -> " . "
  for (size_t i = 0; i < s.size(); ++i) {
    uint32_t c = s[i];
    if (c == U'\n' || c == U'\r' || c == U'\t') continue;
    if (c == U'.') {
      while (i + 1 < s.size() && (s[i + 1] == U'.' || s[i + 1] == U'\n' || s[i + 1] == U'\r' || s[i + 1] == U'\t'))
        ++i;
      t += U" . ";
      continue;
    }
    t.push_back(c);
  }
  // " ".join(RGX.sub(" ", w.strip().lower()) for w in t.split(" ")), then \s+ -> " "
  U32 u;
  size_t start = 0;
  for (size_t i = 0; i <= t.size(); ++i) {
    if (i < t.size() && t[i] != U' ') continue;
    size_t wb = start, we = i;
    while (wb < we && py_space(t[wb])) ++wb;
    while (we > wb && py_space(t[we - 1])) --we;
    if (start > 0) u.push_back(U' ');
    for (size_t k = wb; k < we; ++k) {
      uint32_t c = lower_cp(t[k]);
      u.push_back(w2v_keep(c) ? c : U' ');
    }
    start = i + 1;
  }
  cps.clear();
  bool prev_space = false;
  for (uint32_t c : u) {
    bool sp = py_space(c);
    if (sp && prev_space) continue;
    cps.push_back(sp ? (uint32_t)' ' : c);
    prev_space = sp;
  }
}

inline uint32_t fnv1a(const char* p, size_t n) {
  uint32_t h = 0x811C9DC5u;
  for (size_t i = 0; i < n; ++i) { h ^= (unsigned char)p[i]; h *= 0x01000193u; }
  return h;
}

struct Vocab {
  std::unordered_map<std::string, int32_t> map;
  // char mode: direct code-point -> id table for the BMP (rebuilt after vocabulary edits),
  // so a character costs one array load instead of a std::string hash + compare
  std::vector<int32_t> cp_ids;
  int32_t cp_unk = 0;
  bool cp_valid = false;
  std::mutex mu;
  void add(const char* tok, int32_t id) {
    std::lock_guard<std::mutex> g(mu);
    map[std::string(tok)] = id;
    cp_valid = false;
  }
  void build_cp_table(int32_t unk) {
    std::lock_guard<std::mutex> g(mu);
    if (cp_valid && cp_unk == unk) return;
    cp_ids.assign(0x10000, unk);
    std::vector<uint32_t> cps;
    for (const auto& kv : map) {
      decode_utf8(kv.first.data(), kv.first.size(), cps);
      if (cps.size() == 1 && cps[0] < 0x10000) cp_ids[cps[0]] = kv.second;
    }
    cp_unk = unk;
    cp_valid = true;
  }
};

struct Spec {
  int mode;        // 0 word, 1 ngram, 2 char
  bool html;       // HTML / word2vec normalisation before clean_str (cfg.html_normalize)
  int length;      // cutoff == pad length
  const Vocab* vocab;
  int hash_size;   // > 0 => hashing
  int unk_id;
  int pad_id;
};

// Thread-local scratch for one text.
struct Scratch {
  std::vector<uint32_t> cps;
  std::string utf8;
  std::vector<uint32_t> off;  // byte offset of each code point (+ sentinel)
  std::string key;
  size_t first = 0;           // index in cps of the first code point after the leading strip
};

inline int32_t token_id(const Spec& sp, const char* p, size_t n, Scratch& sc) {
  if (sp.hash_size > 0) return (int32_t)(1 + fnv1a(p, n) % (uint32_t)(sp.hash_size - 1));
  sc.key.assign(p, n);
  auto it = sp.vocab->map.find(sc.key);
  return it == sp.vocab->map.end() ? sp.unk_id : it->second;
}

// clean_str: replace non-kept code points by ' ', strip ' '/'\n', lower-case (after the
// optional HTML normalisation of the raw text).
void clean(const char* s, size_t n, Scratch& sc, bool html = false) {
  decode_utf8(s, n, sc.cps);
  if (html) html_normalize(sc.cps);
  for (auto& c : sc.cps) c = keep_cp(c) ? c : (uint32_t)' ';
  size_t b = 0, e = sc.cps.size();
  auto ws = [](uint32_t c) { return c == ' ' || c == '\n'; };
  while (b < e && ws(sc.cps[b])) ++b;
  while (e > b && ws(sc.cps[e - 1])) --e;
  sc.first = b;
  sc.utf8.clear();
  sc.off.clear();
  for (size_t i = b; i < e; ++i) {
    sc.off.push_back((uint32_t)sc.utf8.size());
    encode_cp(lower_cp(sc.cps[i]), sc.utf8);
  }
  sc.off.push_back((uint32_t)sc.utf8.size());
}

void featurize_one(const char* s, size_t n, const Spec& sp, int32_t* out, Scratch& sc) {
  clean(s, n, sc, sp.html);
  const size_t ncp = sc.off.size() - 1;
  const char* u = sc.utf8.data();
  int t = 0;
  if (sp.mode == 0) {  // word: split on every single ' '
    size_t start = 0;
    for (size_t i = 0; i <= sc.utf8.size() && t < sp.length; ++i) {
      if (i == sc.utf8.size() || u[i] == ' ') {
        out[t++] = token_id(sp, u + start, i - start, sc);
        start = i + 1;
      }
    }
  } else if (sp.mode == 1) {  // overlapping 3-grams of code points
    for (size_t i = 0; i + 3 <= ncp && t < sp.length; ++i)
      out[t++] = token_id(sp, u + sc.off[i], sc.off[i + 3] - sc.off[i], sc);
  } else if (sp.hash_size == 0) {  // char, exact vocabulary: BMP code points by table
    const int32_t* tab = sp.vocab->cp_ids.data();
    for (size_t i = 0; i < ncp && t < sp.length; ++i) {
      const uint32_t c = lower_cp(sc.cps[sc.first + i]);
      out[t++] = c < 0x10000 ? tab[c] : token_id(sp, u + sc.off[i], sc.off[i + 1] - sc.off[i], sc);
    }
  } else {  // char, hashed
    for (size_t i = 0; i < ncp && t < sp.length; ++i)
      out[t++] = token_id(sp, u + sc.off[i], sc.off[i + 1] - sc.off[i], sc);
  }
  for (; t < sp.length; ++t) out[t] = sp.pad_id;
}

template <class F>
void parallel_for(int n, int nthreads, F&& f) {
  if (nthreads <= 1 || n < 2) {
    Scratch sc;
    for (int i = 0; i < n; ++i) f(i, sc);
    return;
  }
  nthreads = std::min(nthreads, n);
  std::atomic<int> next{0};
  std::vector<std::thread> ts;
  for (int k = 0; k < nthreads; ++k)
    ts.emplace_back([&] {
      Scratch sc;
      for (;;) {
        int i = next.fetch_add(1);
        if (i >= n) break;
        f(i, sc);
      }
    });
  for (auto& t : ts) t.join();
}

// ---------------------------------------------------------------- mini JSON --
struct JsonCursor {
  const char* p;
  const char* e;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) ++p; }
};

bool parse_hex4(const char* p, uint32_t& v) {
  v = 0;
  for (int i = 0; i < 4; ++i) {
    char c = p[i];
    v <<= 4;
    if (c >= '0' && c <= '9') v |= c - '0';
    else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
    else return false;
  }
  return true;
}

bool parse_string(JsonCursor& c, std::string* out) {
  c.ws();
  if (c.p >= c.e || *c.p != '"') return false;
  ++c.p;
  if (out) out->clear();
  while (c.p < c.e) {
    char ch = *c.p++;
    if (ch == '"') return true;
    if (ch != '\\') { if (out) out->push_back(ch); continue; }
    if (c.p >= c.e) return false;
    char esc = *c.p++;
    switch (esc) {
      case '"': case '\\': case '/': if (out) out->push_back(esc); break;
      case 'b': if (out) out->push_back('\b'); break;
      case 'f': if (out) out->push_back('\f'); break;
      case 'n': if (out) out->push_back('\n'); break;
      case 'r': if (out) out->push_back('\r'); break;
      case 't': if (out) out->push_back('\t'); break;
      case 'u': {
        uint32_t v;
        if (c.e - c.p < 4 || !parse_hex4(c.p, v)) return false;
        c.p += 4;
        if (v >= 0xD800 && v < 0xDC00 && c.e - c.p >= 6 && c.p[0] == '\\' && c.p[1] == 'u') {
          uint32_t lo;
          if (parse_hex4(c.p + 2, lo) && lo >= 0xDC00 && lo < 0xE000) {
            v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
            c.p += 6;
          }
        }
        if (out) encode_cp(v, *out);
        break;
      }
      default: return false;
    }
  }
  return false;
}

bool skip_value(JsonCursor& c);

bool skip_container(JsonCursor& c, char open, char close) {
  ++c.p;
  c.ws();
  if (c.p < c.e && *c.p == close) { ++c.p; return true; }
  for (;;) {
    if (open == '{') {
      if (!parse_string(c, nullptr)) return false;
      c.ws();
      if (c.p >= c.e || *c.p != ':') return false;
      ++c.p;
    }
    if (!skip_value(c)) return false;
    c.ws();
    if (c.p >= c.e) return false;
    if (*c.p == ',') { ++c.p; continue; }
    if (*c.p == close) { ++c.p; return true; }
    return false;
  }
}

bool skip_value(JsonCursor& c) {
  c.ws();
  if (c.p >= c.e) return false;
  char ch = *c.p;
  if (ch == '"') return parse_string(c, nullptr);
  if (ch == '{') return skip_container(c, '{', '}');
  if (ch == '[') return skip_container(c, '[', ']');
  while (c.p < c.e && *c.p != ',' && *c.p != '}' && *c.p != ']' && *c.p != ' ' && *c.p != '\n') ++c.p;
  return true;
}

struct Record {
  std::string q, pos;
  std::vector<std::string> neg;
  bool has_q = false, has_pos = false, has_neg = false;
};

// Parse {'q': str, 'doc_corr': str, 'doc_incorr': [str...]}; other keys skipped.
bool parse_record(const char* b, const char* e, Record& r) {
  JsonCursor c{b, e};
  r.has_q = r.has_pos = r.has_neg = false;
  r.neg.clear();
  c.ws();
  if (c.p >= c.e || *c.p != '{') return false;
  ++c.p;
  std::string key;
  c.ws();
  if (c.p < c.e && *c.p == '}') return false;
  for (;;) {
    if (!parse_string(c, &key)) return false;
    c.ws();
    if (c.p >= c.e || *c.p != ':') return false;
    ++c.p;
    c.ws();
    if (key == "q" && c.p < c.e && *c.p == '"') {
      if (!parse_string(c, &r.q)) return false;
      r.has_q = true;
    } else if (key == "doc_corr" && c.p < c.e && *c.p == '"') {
      if (!parse_string(c, &r.pos)) return false;
      r.has_pos = true;
    } else if (key == "doc_incorr" && c.p < c.e && *c.p == '[') {
      ++c.p;
      c.ws();
      r.has_neg = true;
      if (c.p < c.e && *c.p == ']') { ++c.p; }
      else {
        for (;;) {
          c.ws();
          if (c.p < c.e && *c.p == '"') {
            r.neg.emplace_back();
            if (!parse_string(c, &r.neg.back())) return false;
          } else if (!skip_value(c)) return false;
          c.ws();
          if (c.p >= c.e) return false;
          if (*c.p == ',') { ++c.p; continue; }
          if (*c.p == ']') { ++c.p; break; }
          return false;
        }
      }
    } else if (!skip_value(c)) {
      return false;
    }
    c.ws();
    if (c.p >= c.e) return false;
    if (*c.p == ',') { ++c.p; continue; }
    if (*c.p == '}') return true;
    return false;
  }
}

struct Dataset {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  std::vector<int64_t> begin, end;  // valid rows only
  int64_t skipped = 0;
  int num_neg = 3;
};

}  // namespace

extern "C" {

void* pv_vocab_new() { return new Vocab(); }
void pv_vocab_free(void* v) { delete (Vocab*)v; }
void pv_vocab_add(void* v, const char* tok, int32_t id) { ((Vocab*)v)->add(tok, id); }
int64_t pv_vocab_size(void* v) { return (int64_t)((Vocab*)v)->map.size(); }

// texts: n NUL-terminated UTF-8 strings. out: n x length int32.
int pv_featurize(const char** texts, int n, int mode, int length, void* vocab, int hash_size, int unk_id,
                 int pad_id, int32_t* out, int nthreads) {
  const bool html = (mode & 4) != 0;  // bit 2: HTML normalisation
  mode &= 3;
  if (mode > 2 || length <= 0) return -1;
  if (hash_size <= 1 && !vocab) return -2;
  Spec sp{mode, html, length, (const Vocab*)vocab, hash_size > 1 ? hash_size : 0, unk_id, pad_id};
  if (mode == 2 && sp.hash_size == 0) ((Vocab*)vocab)->build_cp_table(unk_id);
  parallel_for(n, nthreads, [&](int i, Scratch& sc) {
    featurize_one(texts[i], strlen(texts[i]), sp, out + (int64_t)i * length, sc);
  });
  return 0;
}

// Cleaned text (for tests): writes up to cap bytes, returns the full length.
int64_t pv_clean_str(const char* s, char* out, int64_t cap) {
  Scratch sc;
  clean(s, strlen(s), sc);
  int64_t n = (int64_t)sc.utf8.size();
  if (cap > 0) {
    int64_t m = n < cap - 1 ? n : cap - 1;
    memcpy(out, sc.utf8.data(), (size_t)m);
    out[m] = 0;
  }
  return n;
}

// HTML / word2vec normalisation of one line (tests: parity with data/text.py)
int64_t pv_normalize_html(const char* s, char* out, int64_t cap) {
  std::vector<uint32_t> cps;
  decode_utf8(s, strlen(s), cps);
  html_normalize(cps);
  std::string o;
  for (uint32_t c : cps) encode_cp(c, o);
  int64_t n = (int64_t)o.size();
  if (cap > 0) {
    int64_t m = n < cap - 1 ? n : cap - 1;
    memcpy(out, o.data(), (size_t)m);
    out[m] = 0;
  }
  return n;
}

void* pv_dataset_open(const char* path, int num_neg, int nthreads) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0) { close(fd); return nullptr; }
  auto* ds = new Dataset();
  ds->fd = fd;
  ds->size = (size_t)st.st_size;
  ds->num_neg = num_neg;
  if (ds->size > 0) {
    void* m = mmap(nullptr, ds->size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) { close(fd); delete ds; return nullptr; }
    ds->data = (const char*)m;
  }
  // line boundaries
  std::vector<int64_t> lb, le;
  size_t s = 0;
  for (size_t i = 0; i <= ds->size; ++i) {
    if (i == ds->size || ds->data[i] == '\n') {
      if (i > s) { lb.push_back((int64_t)s); le.push_back((int64_t)i); }
      s = i + 1;
    }
  }
  // validate in parallel (rows whose doc_incorr length != num_neg are skipped,
  // dssm_cnn_v2/data_helpers.py:163,193-194)
  std::vector<char> ok(lb.size(), 0);
  parallel_for((int)lb.size(), nthreads, [&](int i, Scratch&) {
    Record r;
    ok[i] = parse_record(ds->data + lb[i], ds->data + le[i], r) && r.has_q && r.has_pos && r.has_neg &&
            (int)r.neg.size() == num_neg;
  });
  for (size_t i = 0; i < lb.size(); ++i) {
    if (ok[i]) { ds->begin.push_back(lb[i]); ds->end.push_back(le[i]); }
    else ds->skipped++;
  }
  return ds;
}

int64_t pv_dataset_size(void* h) { return (int64_t)((Dataset*)h)->begin.size(); }
int64_t pv_dataset_skipped(void* h) { return ((Dataset*)h)->skipped; }

void pv_dataset_close(void* h) {
  auto* ds = (Dataset*)h;
  if (!ds) return;
  if (ds->data) munmap((void*)ds->data, ds->size);
  if (ds->fd >= 0) close(ds->fd);
  delete ds;
}

// Featurize rows[0..n) into q_out (n x qlen) and d_out (n x (1+J) x dlen): pos first, then negatives.
int pv_dataset_batch(void* h, const int64_t* rows, int n, int mode, int qlen, int dlen, void* vocab,
                     int hash_size, int unk_id, int pad_id, int32_t* q_out, int32_t* d_out, int nthreads) {
  auto* ds = (Dataset*)h;
  const int J = ds->num_neg;
  const bool html = (mode & 4) != 0;
  mode &= 3;
  if (mode > 2) return -3;
  if (mode == 2 && hash_size <= 1 && vocab) ((Vocab*)vocab)->build_cp_table(unk_id);
  Spec sq{mode, html, qlen, (const Vocab*)vocab, hash_size > 1 ? hash_size : 0, unk_id, pad_id};
  Spec sd{mode, html, dlen, (const Vocab*)vocab, hash_size > 1 ? hash_size : 0, unk_id, pad_id};
  std::atomic<int> err{0};
  parallel_for(n, nthreads, [&](int i, Scratch& sc) {
    int64_t r = rows[i];
    if (r < 0 || r >= (int64_t)ds->begin.size()) { err = -1; return; }
    Record rec;
    if (!parse_record(ds->data + ds->begin[r], ds->data + ds->end[r], rec)) { err = -2; return; }
    featurize_one(rec.q.data(), rec.q.size(), sq, q_out + (int64_t)i * qlen, sc);
    int32_t* d = d_out + (int64_t)i * (1 + J) * dlen;
    featurize_one(rec.pos.data(), rec.pos.size(), sd, d, sc);
    for (int j = 0; j < J; ++j) featurize_one(rec.neg[j].data(), rec.neg[j].size(), sd, d + (int64_t)(1 + j) * dlen, sc);
  });
  return err.load();
}

// Raw strings of one row (for vocab building in Python): returns bytes needed.
int64_t pv_dataset_row_text(void* h, int64_t row, int field, char* out, int64_t cap) {
  auto* ds = (Dataset*)h;
  if (row < 0 || row >= (int64_t)ds->begin.size()) return -1;
  Record rec;
  if (!parse_record(ds->data + ds->begin[row], ds->data + ds->end[row], rec)) return -2;
  const std::string* s = field == 0 ? &rec.q : field == 1 ? &rec.pos
                         : (field - 2 < (int)rec.neg.size() ? &rec.neg[field - 2] : nullptr);
  if (!s) return -3;
  int64_t n = (int64_t)s->size();
  if (cap > n) { memcpy(out, s->data(), (size_t)n); out[n] = 0; }
  return n;
}

}  // extern "C"
