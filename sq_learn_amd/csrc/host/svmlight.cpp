// SVMlight / libsvm text parser (reference
// ``datasets/_svmlight_format_fast.pyx``): one pass over an in-memory byte
// buffer into CSR arrays, labels (or sorted multilabel tuples) and query
// ids.  Same format rules as the reference: '#' starts a comment, blank
// lines are skipped, an optional ``qid:<int>`` follows the target, feature
// indices must be strictly increasing, index < 0 (or 0 when one-based) is
// an error, and a multilabel line whose first token holds ':' has no
// labels.  ``offset``/``length`` select a byte range the way the reference
// does: skip the (possibly partial) line at ``offset``, stop after the line
// that ends past ``offset + length``.
#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "host.h"

namespace {

struct Parsed {
  std::vector<double> labels;
  std::vector<long long> label_off{0};   // multilabel: labels[off[i]:off[i+1]]
  std::vector<long long> qids;
  std::vector<double> data;
  std::vector<long long> indices;
  std::vector<long long> indptr{0};
  std::string error;
};

bool parse_double(const char* b, const char* e, double* out) {
  std::string s(b, e);
  char* end = nullptr;
  errno = 0;
  *out = std::strtod(s.c_str(), &end);
  return end == s.c_str() + s.size() && !s.empty();
}

bool parse_ll(const char* b, const char* e, long long* out) {
  std::string s(b, e);
  char* end = nullptr;
  errno = 0;
  *out = std::strtoll(s.c_str(), &end, 10);
  return end == s.c_str() + s.size() && !s.empty() && errno == 0;
}

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// returns false (with p->error set) on malformed input
bool parse_line(const char* b, const char* e, Parsed* p, bool multilabel, bool zero_based,
                bool query_id) {
  const char* h = static_cast<const char*>(std::memchr(b, '#', e - b));
  if (h) e = h;
  std::vector<std::pair<const char*, const char*>> tok;
  for (const char* c = b; c < e;) {
    while (c < e && is_space(*c)) ++c;
    const char* s = c;
    while (c < e && !is_space(*c)) ++c;
    if (c > s) tok.push_back({s, c});
  }
  if (tok.empty()) return true;
  size_t first_feat = 1;
  if (multilabel) {
    const auto [tb, te] = tok[0];
    if (std::memchr(tb, ':', te - tb)) {
      first_feat = 0;   // no labels on this line
    } else {
      std::vector<double> ls;
      const char* s = tb;
      for (const char* c = tb; c <= te; ++c) {
        if (c == te || *c == ',') {
          double v;
          if (!parse_double(s, c, &v)) {
            p->error = "could not convert string to float: '" + std::string(s, c) + "'";
            return false;
          }
          ls.push_back(v);
          s = c + 1;
        }
      }
      std::sort(ls.begin(), ls.end());
      p->labels.insert(p->labels.end(), ls.begin(), ls.end());
    }
    p->label_off.push_back((long long)p->labels.size());
  } else {
    double v;
    if (!parse_double(tok[0].first, tok[0].second, &v)) {
      p->error = "could not convert string to float: '" +
                 std::string(tok[0].first, tok[0].second) + "'";
      return false;
    }
    p->labels.push_back(v);
  }
  if (first_feat < tok.size() && tok[first_feat].second - tok[first_feat].first >= 3 &&
      std::strncmp(tok[first_feat].first, "qid", 3) == 0) {
    const char* c = static_cast<const char*>(
        std::memchr(tok[first_feat].first, ':', tok[first_feat].second - tok[first_feat].first));
    if (query_id) {
      long long q = 0;
      if (!c || !parse_ll(c + 1, tok[first_feat].second, &q)) {
        p->error = "invalid qid";
        return false;
      }
      p->qids.push_back(q);
    }
    ++first_feat;
  }
  long long prev = -1;
  for (size_t t = first_feat; t < tok.size(); ++t) {
    const auto [tb, te] = tok[t];
    const char* c = static_cast<const char*>(std::memchr(tb, ':', te - tb));
    if (!c) {
      p->error = "not enough values to unpack (expected 2, got 1)";
      return false;
    }
    long long idx;
    double v;
    if (!parse_ll(tb, c, &idx)) {
      p->error = "invalid literal for int() with base 10: '" + std::string(tb, c) + "'";
      return false;
    }
    if (idx < 0 || (!zero_based && idx == 0)) {
      p->error = "Invalid index " + std::to_string(idx) + " in SVMlight/LibSVM data file.";
      return false;
    }
    if (idx <= prev) {
      p->error = "Feature indices in SVMlight/LibSVM data file should be sorted and unique.";
      return false;
    }
    if (!parse_double(c + 1, te, &v)) {
      p->error = "could not convert string to float: '" + std::string(c + 1, te) + "'";
      return false;
    }
    p->indices.push_back(idx);
    p->data.push_back(v);
    prev = idx;
  }
  p->indptr.push_back((long long)p->data.size());
  return true;
}

}  // namespace

template <class T>
static void copy_out(T* dst, const std::vector<T>& src) {
  if (dst && !src.empty()) std::memcpy(dst, src.data(), src.size() * sizeof(T));
}

extern "C" {

void* sqh_svml_parse(const char* buf, long long len, int multilabel, int zero_based,
                     int query_id, long long offset, long long length) {
  auto* p = new Parsed();
  long long pos = 0;
  if (offset > 0) {
    pos = offset;
    while (pos < len && buf[pos] != '\n') ++pos;   // drop the partial line
    if (pos < len) ++pos;
  }
  const long long stop = length > 0 ? offset + length : -1;
  while (pos < len) {
    long long e = pos;
    while (e < len && buf[e] != '\n') ++e;
    if (!parse_line(buf + pos, buf + e, p, multilabel, zero_based, query_id)) break;
    pos = e < len ? e + 1 : len;
    if (stop != -1 && pos > stop) break;
  }
  return p;
}

const char* sqh_svml_error(void* h) {
  auto* p = static_cast<Parsed*>(h);
  return p->error.empty() ? nullptr : p->error.c_str();
}

// sizes: [n_rows, nnz, n_labels_flat, n_qids]
void sqh_svml_sizes(void* h, long long* sizes) {
  auto* p = static_cast<Parsed*>(h);
  sizes[0] = (long long)p->indptr.size() - 1;
  sizes[1] = (long long)p->data.size();
  sizes[2] = (long long)p->labels.size();
  sizes[3] = (long long)p->qids.size();
}

void sqh_svml_copy(void* h, double* labels, long long* label_off, long long* qids, double* data,
                   long long* indices, long long* indptr) {
  auto* p = static_cast<Parsed*>(h);
  copy_out(labels, p->labels);
  copy_out(label_off, p->label_off);
  copy_out(qids, p->qids);
  copy_out(data, p->data);
  copy_out(indices, p->indices);
  copy_out(indptr, p->indptr);
}

void sqh_svml_free(void* h) { delete static_cast<Parsed*>(h); }

}  // extern "C"
