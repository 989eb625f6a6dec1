// Heuristic spatial document graph (host code, C ABI).
//
// Native replacement for the reference's graph construction
//   Graph(...) / Graph._get_adj_matrix   gnn/data_generator/data_process/utils/graph_utils.py:425-834
// as driven by HeuristicGraphBuilder     gnn/data_generator/data_process/heuristic_graph_builder.py:23-83.
// It reproduces the same node set and the same six edge types (lr, rl, tb, bt,
// child, parent), in double precision with the reference's expression order,
// and emits either the collate-layout dense adjacency (N, 6, N) the reference
// stores as fp16, or the typed edge list directly (the §8(f) "emit CSR, not a
// dense (N,6,N)" row): no dense O(N^2) matrix is needed for the GPU path.
//
// Node order follows the reference: text lines, then table cells, then the
// detected rows and columns.  The reference slices its adjacency to the first
// min(#items, #nodes) nodes; callers pass that count as out_n.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "grl.h"

namespace grl {
void set_error(const char* fmt, ...);  // common.hip: thread-local grl_last_error()
}

namespace {

struct Node {
  double x, y, w, h;
  bool is_sub = false;  // text line (a "sub" cell in the reference)
  bool has_text = false;
  std::vector<int> lefts, rights, tops, bottoms;
};

struct Edge {
  int start, end, label;
};

enum { LR = 0, RL = 1, TB = 2, BT = 3, CHILD = 4, PARENT = 5 };

// ranges: (x, len) along one axis
inline bool range_hits(double x1, double l1, double x2, double l2) {
  if (x1 > x2) {
    std::swap(x1, x2);
    std::swap(l1, l2);
  }
  return (x1 + l1) > x2;
}
inline double range_overlap(double x1, double l1, double x2, double l2) {
  if (x1 > x2) {
    std::swap(x1, x2);
    std::swap(l1, l2);
  }
  if (!range_hits(x1, l1, x2, l2)) return 0;
  if ((x1 + l1) > (x2 + l2)) return l2;
  return x1 + l1 - x2;
}
// "horizontal projection" = overlap of y ranges, "vertical" = of x ranges
inline bool hits_y(const Node& a, const Node& b) { return range_hits(a.y, a.h, b.y, b.h); }
inline bool hits_x(const Node& a, const Node& b) { return range_hits(a.x, a.w, b.x, b.w); }
inline double overlap_y(const Node& a, const Node& b) { return range_overlap(a.y, a.h, b.y, b.h); }
inline double overlap_x(const Node& a, const Node& b) { return range_overlap(a.x, a.w, b.x, b.w); }

inline bool contains(const std::vector<int>& v, int x) { return std::find(v.begin(), v.end(), x) != v.end(); }
inline void erase_first(std::vector<int>& v, int x) {
  auto it = std::find(v.begin(), v.end(), x);
  if (it != v.end()) v.erase(it);
}

class LayoutGraph {
 public:
  std::vector<Node> nodes;
  std::vector<int> lines, cells;  // node ids
  std::vector<Edge> edges;
  int n_rows = 0, n_cols = 0;

  // self directly left of other, given the candidate set ref (CellNode.is_left_of)
  bool left_of(int s, int o, const std::vector<int>& ref) const {
    const Node& a = nodes[s];
    const Node& b = nodes[o];
    if (contains(a.rights, o)) return true;
    if (b.x < a.x || !hits_y(a, b)) return false;
    if (overlap_y(a, b) > 0.9 * std::min(a.h, b.h)) {
      if (b.x - a.x < 0.1 * std::min(a.w, b.w)) return true;
    }
    if (ref.empty()) return true;
    for (int c : ref) {  // any cell strictly between the two blocks the link
      const Node& k = nodes[c];
      if (!(hits_y(a, k) && (k.x + k.w) < b.x + b.w * 0.1 && k.x >= (a.x + a.w * 0.8) && hits_y(a, k))) continue;
      if (!(overlap_y(a, k) > std::min(a.h, k.h) / 5)) continue;
      if (overlap_y(k, b) > b.h / 2 || overlap_y(a, k) > std::min(k.h, a.h) * 0.8) return false;
    }
    return true;
  }

  void add(int s, int e, int label) { edges.push_back(Edge{s, e, label}); }

  void build_left_right(const std::vector<int>& group) {
    std::vector<int> order(group);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return nodes[a].y < nodes[b].y; });
    for (int c : order) {
      std::vector<int> collide;
      for (int o : order) {
        if (o == c) continue;
        if (nodes[o].x >= nodes[c].x && hits_y(nodes[c], nodes[o]) &&
            overlap_y(nodes[c], nodes[o]) > std::min(nodes[c].h, nodes[o].h) * 0.4)
          collide.push_back(o);
      }
      for (int o : collide) {
        if (left_of(c, o, collide) && !contains(nodes[c].rights, o)) {
          add(c, o, LR);
          add(o, c, RL);
          nodes[c].rights.push_back(o);
          nodes[o].lefts.push_back(c);
        }
      }
    }
  }

  // get_nearest_line(cr_line, list, "t"): closest line above with text
  int nearest_top(int cur, const std::vector<int>& cand) const {
    const Node& L = nodes[cur];
    int best = -1;
    double dt = 50000;
    for (int o : cand) {
      const Node& c = nodes[o];
      if (!c.has_text) continue;
      const double d = std::min(std::fabs(c.y - L.y - L.h), std::fabs(L.y - c.y - c.h));
      const double hint = std::max(0.0, std::min(c.x + c.w - L.x, L.x + L.w - c.x));
      if (hint <= 0) {
        if (L.y > c.y) continue;
        if (!(d < 0.5 * L.h && L.y + 1.3 * L.h > c.y)) continue;
      }
      double dist = dt + 1;
      if (c.y < L.y) dist = L.y - c.y - c.h;
      if (dist < dt) {
        best = o;
        dt = dist;
      }
    }
    return best;
  }

  void build_top_down(const std::vector<int>& group) {
    std::vector<int> order(group);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return nodes[a].x < nodes[b].x; });
    for (int c : order) {
      const int t = nearest_top(c, order);
      if (t >= 0) {
        add(t, c, TB);
        add(c, t, BT);
        nodes[c].tops.push_back(t);
        nodes[t].bottoms.push_back(c);
      }
    }
  }

  void drop_pair(int c, int cell, int fwd_label, int rev_label) {
    edges.erase(std::remove_if(edges.begin(), edges.end(),
                               [&](const Edge& e) {
                                 return (e.start == c && e.end == cell && e.label == fwd_label) ||
                                        (e.start == cell && e.end == c && e.label == rev_label);
                               }),
                edges.end());
  }

  // keep only the nearest column of left neighbours (_clean_left_right_edges)
  void clean_left_right() {
    for (int cell : lines) {
      Node& me = nodes[cell];
      if (me.lefts.size() <= 1) continue;
      std::vector<int> left(me.lefts);
      std::stable_sort(left.begin(), left.end(), [&](int a, int b) { return nodes[a].x < nodes[b].x; });
      std::vector<int> removes;
      for (int c : left)
        if (nodes[c].x + nodes[c].w > me.x && nodes[c].x > me.x - 0.5 * me.h) removes.push_back(c);
      std::vector<int> kept;
      for (int c : left)
        if (!contains(removes, c)) kept.push_back(c);
      std::vector<std::vector<int>> columns;
      std::vector<int> col;
      for (int c : kept) {
        double its = 0, uni = 100;
        if (!col.empty()) {
          its = overlap_x(nodes[col.back()], nodes[c]);
          uni = std::min(nodes[col.back()].w, nodes[c].w);
        }
        if (its > 0.5 * uni) {
          col.push_back(c);
          continue;
        }
        if (!col.empty()) columns.push_back(col);
        col = {c};
      }
      if (!col.empty()) columns.push_back(col);
      std::vector<int> real = columns.empty() ? std::vector<int>{} : columns.back();
      for (int c : kept)
        if (!contains(real, c)) removes.push_back(c);
      for (int c : removes) {
        erase_first(nodes[c].rights, cell);
        drop_pair(c, cell, LR, RL);
      }
      me.lefts = real;
    }
  }

  // keep only the nearest row of top neighbours (_clean_top_bot_edges)
  void clean_top_bot() {
    for (int cell : lines) {
      Node& me = nodes[cell];
      if (me.tops.size() <= 1) continue;
      std::vector<int> top(me.tops);
      std::stable_sort(top.begin(), top.end(), [&](int a, int b) { return nodes[a].y < nodes[b].y; });
      std::vector<std::vector<int>> rows;
      std::vector<int> row;
      for (int c : top) {
        double its = 0, uni = 10000;
        if (!row.empty()) {
          its = overlap_y(nodes[row.back()], nodes[c]);
          uni = std::min(nodes[row.back()].w, nodes[c].w);
        }
        if (its > 0.5 * uni) {
          row.push_back(c);
          continue;
        }
        if (!row.empty()) rows.push_back(row);
        row = {c};
      }
      if (!row.empty()) rows.push_back(row);
      const std::vector<int>& real = rows.back();
      for (int c : top) {
        if (contains(real, c)) continue;
        erase_first(nodes[c].bottoms, cell);
        drop_pair(c, cell, TB, BT);
      }
      me.tops = real;
    }
  }

  // rows (by_y) / columns of aligned table cells (_detect_row / _detect_column)
  void detect_groups(bool by_y, std::vector<std::vector<int>>& groups) const {
    std::vector<char> used(nodes.size(), 0);
    for (int c : cells) {
      if (used[c]) continue;
      std::vector<int> al{c};
      const Node& a = nodes[c];
      const double pm = by_y ? a.h / 2 : a.w / 4;
      const double sm = by_y ? a.h / 4 : a.w / 6;
      for (int o : cells) {
        if (used[o] || o == c) continue;
        const Node& b = nodes[o];
        const double dp = by_y ? std::fabs(b.y - a.y) : std::fabs(b.x - a.x);
        const double ds = by_y ? std::fabs(b.h - a.h) : std::fabs(b.w - a.w);
        if (dp <= pm && ds <= sm) al.push_back(o);
      }
      for (int o : al) used[o] = 1;
      if (al.size() > 1) groups.push_back(al);
    }
  }

  void build(const GrlLayoutItem* items, int n) {
    // nodes: text lines (input order), then cells; "table" items are dropped
    std::vector<Node> ln, cl;
    for (int i = 0; i < n; ++i) {
      Node nd;
      nd.x = items[i].x1;
      nd.y = items[i].y1;
      nd.w = items[i].x2 - items[i].x1 + 1;
      nd.h = items[i].y2 - items[i].y1 + 1;
      if (items[i].kind == 0) {
        nd.is_sub = true;
        nd.has_text = items[i].has_text != 0;
        ln.push_back(nd);
      } else if (items[i].kind == 1) {
        nd.has_text = false;  // a cell's text is the join of its (never attached) sub-lines
        cl.push_back(nd);
      }
    }
    for (auto& x : ln) {
      lines.push_back((int)nodes.size());
      nodes.push_back(x);
    }
    for (auto& x : cl) {
      cells.push_back((int)nodes.size());
      nodes.push_back(x);
    }
    std::vector<std::vector<int>> rows, cols;
    detect_groups(true, rows);
    detect_groups(false, cols);
    std::vector<int> row_ids, col_ids;
    for (auto& r : rows) {
      Node nd;
      nd.x = 1e300;
      nd.y = 1e300;
      nd.w = 0;
      for (int c : r) {
        nd.x = std::min(nd.x, nodes[c].x);
        nd.y = std::min(nd.y, nodes[c].y);
        nd.w += nodes[c].w;
      }
      nd.h = nodes[r[0]].h;
      row_ids.push_back((int)nodes.size());
      nodes.push_back(nd);
    }
    for (auto& cgrp : cols) {
      Node nd;
      nd.x = 1e300;
      nd.y = 1e300;
      nd.h = 0;
      for (int c : cgrp) {
        nd.x = std::min(nd.x, nodes[c].x);
        nd.y = std::min(nd.y, nodes[c].y);
        nd.h += nodes[c].h;
      }
      nd.w = nodes[cgrp[0]].w;
      col_ids.push_back((int)nodes.size());
      nodes.push_back(nd);
    }
    n_rows = (int)row_ids.size();
    n_cols = (int)col_ids.size();
    for (const std::vector<int>* group : {&lines, &cells}) {
      build_left_right(*group);
      build_top_down(*group);
    }
    for (size_t r = 0; r < rows.size(); ++r)
      for (int c : rows[r]) {
        add(c, row_ids[r], PARENT);
        add(row_ids[r], c, CHILD);
      }
    for (size_t k = 0; k < cols.size(); ++k)
      for (int c : cols[k]) {
        add(c, col_ids[k], PARENT);
        add(col_ids[k], c, CHILD);
      }
    clean_left_right();
    clean_top_bot();
  }
};

// IEEE binary16 bits of a double, round to nearest even (numpy astype(float16)).
uint16_t double_to_half(double d) {
  uint64_t b;
  std::memcpy(&b, &d, 8);
  const uint16_t sign = (uint16_t)((b >> 48) & 0x8000);
  const int exp = (int)((b >> 52) & 0x7FF);
  uint64_t man = b & 0xFFFFFFFFFFFFFull;
  if (exp == 0x7FF) return sign | 0x7C00 | (man ? 0x200 : 0);  // inf / nan
  const int e = exp - 1023 + 15;                                // half exponent
  if (e >= 31) return sign | 0x7C00;                            // overflow
  if (e <= 0) {                                                 // subnormal half (or zero)
    if (e < -10) return sign;
    man |= 1ull << 52;
    const int shift = 52 - 10 + 1 - e;  // bits to drop
    uint64_t q = man >> shift;
    const uint64_t rem = man & ((1ull << shift) - 1), half = 1ull << (shift - 1);
    if (rem > half || (rem == half && (q & 1))) ++q;
    return sign | (uint16_t)q;
  }
  uint64_t q = man >> 42;
  const uint64_t rem = man & ((1ull << 42) - 1), half = 1ull << 41;
  uint32_t out = ((uint32_t)e << 10) | (uint32_t)q;
  if (rem > half || (rem == half && (q & 1))) ++out;  // may carry into the exponent: still correct
  return sign | (uint16_t)out;
}

double rect_gap(const double r1[4], const double r2[4]) {
  const double x1 = r1[0], y1 = r1[1], x1b = r1[2], y1b = r1[3];
  const double x2 = r2[0], y2 = r2[1], x2b = r2[2], y2b = r2[3];
  const bool left = x2b < x1, right = x1b < x2, bottom = y2b < y1, top = y1b < y2;
  auto dist = [](double a, double b, double c, double d) { return std::sqrt((a - c) * (a - c) + (b - d) * (b - d)); };
  if (top && left) return dist(x1, y1b, x2b, y2);
  if (left && bottom) return dist(x1, y1, x2b, y2b);
  if (bottom && right) return dist(x1b, y1, x2, y2b);
  if (right && top) return dist(x1b, y1b, x2, y2);
  if (left) return x1 - x2b;
  if (right) return x2 - x1b;
  if (bottom) return y1 - y2b;
  if (top) return y2 - y1b;
  return 0.0;
}

int check_items(const GrlLayoutItem* items, int32_t n) {
  if (n < 0 || (n > 0 && !items)) {
    grl::set_error("%s", "layout graph: bad item array");
    return GRL_E_INVALID;
  }
  return GRL_OK;
}

}  // namespace

extern "C" int grl_layout_graph_size(const GrlLayoutItem* items, int32_t n, int32_t* out_n) {
  if (int rc = check_items(items, n)) return rc;
  if (!out_n) {
    grl::set_error("%s", "grl_layout_graph_size: out_n is NULL");
    return GRL_E_INVALID;
  }
  LayoutGraph g;
  g.build(items, n);
  *out_n = std::min<int32_t>(n, (int32_t)g.nodes.size());
  return GRL_OK;
}

extern "C" int grl_layout_graph_dense(const GrlLayoutItem* items, int32_t n, int32_t edge_type, int32_t out_n,
                                      uint16_t* adj_half) {
  if (int rc = check_items(items, n)) return rc;
  if (edge_type < 0 || edge_type > 2 || out_n < 0 || (out_n > 0 && !adj_half)) {
    grl::set_error("%s", "grl_layout_graph_dense: bad edge_type/out_n/adj");
    return GRL_E_INVALID;
  }
  LayoutGraph g;
  g.build(items, n);
  const int N = (int)g.nodes.size();
  if (out_n > N) {
    grl::set_error("%s", "grl_layout_graph_dense: out_n exceeds the node count");
    return GRL_E_INVALID;
  }
  const int L = 6;
  std::memset(adj_half, 0, sizeof(uint16_t) * (size_t)out_n * L * out_n);
  auto put = [&](int i, int t, int j, uint16_t v) {
    if (i < out_n && j < out_n) adj_half[((size_t)i * L + t) * out_n + j] = v;
  };
  const uint16_t one = 0x3C00;
  if (edge_type == 0) {  // normal_binary
    for (const Edge& e : g.edges) put(e.start, e.label, e.end, one);
    return GRL_OK;
  }
  // fully connected variants over all nodes, values from scaled box gaps
  double max_x = -1e300, max_y = -1e300, min_x = 1e300, min_y = 1e300;
  for (const Node& nd : g.nodes) {
    max_x = std::max(max_x, nd.x + nd.w);
    max_y = std::max(max_y, nd.y + nd.h);
    min_x = std::min(min_x, nd.x);
    min_y = std::min(min_y, nd.y);
  }
  const double dx = std::fabs(max_x - min_x), dy = std::fabs(max_y - min_y);
  auto scaled = [&](const Node& nd, double r[4]) {
    r[0] = (nd.x - min_x) / dx;
    r[1] = (nd.y - min_y) / dy;
    r[2] = (nd.x + nd.w - min_x) / dx;
    r[3] = (nd.y + nd.h - min_y) / dy;
  };
  for (int i = 0; i < N; ++i) {
    for (int j = i; j < N; ++j) {
      uint16_t v = one;
      if (i != j && edge_type == 1) {
        double ri[4], rj[4];
        scaled(g.nodes[i], ri);
        scaled(g.nodes[j], rj);
        const double ed = std::fabs(rect_gap(ri, rj));
        const double s = 1 - (ed / std::sqrt(2.0));
        v = double_to_half(s * s);
      }
      for (int t = 0; t < L; ++t) {
        put(i, t, j, v);
        put(j, t, i, v);
      }
    }
  }
  return GRL_OK;
}

extern "C" int grl_layout_graph_edges(const GrlLayoutItem* items, int32_t n, int32_t out_n, int32_t* edges,
                                      int64_t capacity, int64_t* count) {
  if (int rc = check_items(items, n)) return rc;
  if (!count || out_n < 0 || (capacity > 0 && !edges)) {
    grl::set_error("%s", "grl_layout_graph_edges: bad arguments");
    return GRL_E_INVALID;
  }
  LayoutGraph g;
  g.build(items, n);
  std::vector<int64_t> keys;
  keys.reserve(g.edges.size());
  for (const Edge& e : g.edges)
    if (e.start < out_n && e.end < out_n) keys.push_back(((int64_t)e.start * 6 + e.label) * out_n + e.end);
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  *count = (int64_t)keys.size();
  if ((int64_t)keys.size() > capacity) return GRL_OK;  // caller re-calls with enough room
  for (size_t i = 0; i < keys.size(); ++i) {
    const int64_t k = keys[i];
    edges[3 * i + 0] = (int32_t)(k / (6LL * out_n));
    edges[3 * i + 1] = (int32_t)((k / out_n) % 6);
    edges[3 * i + 2] = (int32_t)(k % out_n);
  }
  return GRL_OK;
}
