// Native planner of MemorySystem.consolidate_batch (lazzaro_amd/core/batch_plan.py
// holds the reference Python implementation and the design notes): a host
// simulation of B sequential end_conversation calls (reference
// memory_system.py:580-649, :651-933) from one scan's candidate lists --
// dedupe (the store's L2 top-1), insert, chain / within-shard / cross-memory
// links, buffer-limit eviction over a pool, super-node creation, decay +
// prune -- producing the segments the Python side applies to the device
// graph. Rounding follows the device kernels operation by operation
// (tg_decay_kernel's decay_sal, tg_importance_kernel), so the plan is the
// sequential result bit for bit. Compiled with -ffp-contract=off.
#include "batch_plan.h"

#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <map>
#include <set>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

namespace {

using i64 = int64_t;
template <class T>
using arr = py::array_t<T, py::array::c_style | py::array::forcecast>;

constexpr float kSalFloor = 0.2f;

inline float decay_sal(float s, float keep) {
  if (!(s > kSalFloor)) return kSalFloor;
  const float d = s - kSalFloor;
  const float m = d * keep;
  return kSalFloor + m;
}

// importance = (a + b) + c with a = 0.5 sal, b from the access count, c from
// the recency -- rounded op by op like tg_importance_kernel (the GPU verifies
// the plan's eviction events against it bit for bit). b and c only change
// when a row is touched, so the planner keeps them per row (imp_b / imp_c)
// and each eviction pass costs one multiply and two adds per row.
inline double imp_b(i64 acc) { return std::min(1.0, (double)acc / 10.0) * 0.3; }
inline double imp_c(double last, double now) {
  const double days = (now - last) / 86400.0;
  return (1.0 / (1.0 + days)) * 0.2;
}
inline double importance_bc(float sal, double b, double c) { return ((double)sal * 0.5 + b) + c; }
inline double importance(float sal, i64 acc, double last, double now) {
  return importance_bc(sal, imp_b(acc), imp_c(last, now));
}

struct Super {
  i64 code, key;
  int conv;
  std::vector<i64> children;
  std::vector<double> cos;
  double n2;
};

struct Seg {
  int c0, c1;
  std::vector<std::pair<int, int>> inserts;  // (0 fact / 1 super, index)
  std::vector<int> edges;
  std::vector<i64> victims;
  std::unordered_set<i64> touched;
  bool consolidate = false, cluster = false;
  // filled at close
  std::vector<double> ins_sal, ins_last, tch_sal, tch_last;
  std::vector<i64> ins_acc, tch_rows, tch_acc;
  std::vector<float> edge_w;
};

struct Cand {
  double v;
  i64 r;
};

class Planner {
 public:
  // facts
  int M = 0, K = 0, S = 0;
  std::vector<i64> ct, code;
  std::vector<float> sal_in;
  std::vector<double> gs, ss, sup_cos, sup_n2, qnorm, fact_n2;
  arr<double> Sarr;            // the F x F fact block, read in place (8 MB per 1,024-fact batch)
  const double* Sp = nullptr;
  std::vector<i64> gr, sr, sup_rows;
  // graph
  i64 n0 = 0, node_count = 0, max_buffer = 0;
  std::vector<i64> shard_count;
  std::set<i64> super_codes;
  double sthr = 0, now = 0, dedupe_thr = 0.95, link_thr = 0.5, link_scale = 0.8;
  bool ref_h = true, has_thr = true;
  float thr = 0.5f, keep = 0.99f, chain_w = 0.5f;
  int link_k = 3;
  py::function pre_members, super_cos_fn, fallback_fn;
  // node state
  std::vector<i64> row, acc, ncode;
  std::vector<float> sal;
  std::vector<double> last, n2, ib, ic;  // ib / ic: imp_b(acc), imp_c(last) per row
  std::vector<uint8_t> sup, alive, cand;
  std::unordered_map<i64, int> loc;
  // batch
  std::vector<i64> fact_key, dup_of;
  std::vector<uint8_t> fact_live;
  std::unordered_map<i64, int> key_fact;
  std::unordered_map<i64, int> evicted;
  std::vector<i64> evicted_pre;
  std::vector<Super> supers;
  std::vector<i64> e_src, e_dst, e_code;
  std::vector<int> e_conv;
  std::vector<float> e_w;
  std::vector<uint8_t> e_alive;
  std::unordered_map<i64, std::vector<int>> inc;
  std::vector<std::tuple<int, double, i64, i64>> events;
  int decays = 0;
  i64 next_row = 0;
  std::map<std::string, i64> stats{{"dup", 0},      {"inserted", 0},    {"linked", 0}, {"cross_links", 0},
                                   {"pruned_new", 0}, {"evicted", 0}, {"fallbacks", 0}};
  std::vector<Seg> segs;
  Seg* seg = nullptr;
  int conv_first = 0;  // first fact of the current conversation (facts are in conversation order)
  // near[j]: the facts of earlier conversations whose similarity to fact j is
  // above the link threshold, in fact order -- the only fact x fact entries
  // cands() can use (one O(M^2) pass instead of one per cands() call)
  std::vector<std::vector<std::pair<int, double>>> near;

  void build_near() {
    near.assign(M, {});
    for (int j = 0; j < M; ++j) {
      const double* srow = Sp + (size_t)j * M;
      for (int i = 0; i < M && ct[i] < ct[j]; ++i)
        if (srow[i] > link_thr) near[j].emplace_back(i, srow[i]);
    }
  }

  bool present(i64 r) const { return evicted.find(r) == evicted.end(); }

  int add_state(i64 r, float s, i64 c, bool is_sup, double nn2) {
    const int i = (int)row.size();
    row.push_back(r);
    sal.push_back(s);
    acc.push_back(0);
    last.push_back(now);
    ib.push_back(imp_b(0));
    ic.push_back(imp_c(now, now));
    ncode.push_back(c);
    sup.push_back(is_sup);
    alive.push_back(1);
    cand.push_back(!is_sup);
    n2.push_back(nn2);
    loc[r] = i;
    return i;
  }

  void cands(int j, bool same, int c, std::vector<Cand>& out) {
    out.clear();
    const double* s = (same ? ss.data() : gs.data()) + (size_t)j * K;
    const i64* r = (same ? sr.data() : gr.data()) + (size_t)j * K;
    for (int t = 0; t < K; ++t)
      if (r[t] >= 0 && s[t] > link_thr && present(r[t])) out.push_back({s[t], r[t]});
    const bool full = K > 0 && r[K - 1] >= 0 && s[K - 1] > link_thr;
    if (full && (int)out.size() < link_k + 1) {
      py::gil_scoped_acquire gil;  // (run() releases the GIL; the callbacks are Python)
      py::array_t<i64> ev(evicted_pre.size(), evicted_pre.data());
      py::tuple res = fallback_fn(j, ev, same);
      auto s2 = py::cast<arr<double>>(res[0]);
      auto r2 = py::cast<arr<i64>>(res[1]);
      ++stats["fallbacks"];
      out.clear();
      for (py::ssize_t t = 0; t < r2.size(); ++t)
        if (r2.data()[t] >= 0 && s2.data()[t] > link_thr && present(r2.data()[t]))
          out.push_back({s2.data()[t], r2.data()[t]});
    }
    for (const auto& [i, v] : near[j]) {  // kept facts of earlier conversations above the link threshold
      if (!fact_live[i] || (same && code[i] != code[j])) continue;
      out.push_back({v, fact_key[i]});
    }
    std::sort(out.begin(), out.end(), [](const Cand& a, const Cand& b) { return a.v > b.v || (a.v == b.v && a.r < b.r); });
  }

  std::vector<int> dedupe(const std::vector<int>& jj, int c) {
    std::vector<int> kept;
    std::map<i64, std::vector<int>> pending;
    std::vector<Cand> cl;
    for (int j : jj) {
      const double qn = qnorm[j];
      double bl2 = -INFINITY, bcos = -INFINITY;
      i64 br = -1;
      auto offer = [&](double cs, i64 r, double nn2) {
        const double l2 = 2.0 * qn * cs * std::sqrt(nn2) - nn2;
        if (l2 > bl2 || (l2 == bl2 && r < br)) {
          bl2 = l2;
          br = r;
          bcos = cs;
        }
      };
      cands(j, false, c, cl);
      if (!cl.empty()) offer(cl[0].v, cl[0].r, n2[loc.at(cl[0].r)]);
      for (int si = 0; si < S; ++si) offer(sup_cos[(size_t)j * S + si], sup_rows[si], sup_n2[si]);
      for (auto& sp : supers)
        if (sp.conv < ct[j]) offer(sp.cos[j], sp.key, sp.n2);
      if (br >= 0 && bcos > dedupe_thr) {
        pending[br].push_back(j);
        dup_of[j] = br;
        ++stats["dup"];
      } else {
        kept.push_back(j);
      }
    }
    for (auto& [r, js] : pending) {
      const int i = loc.at(r);
      float m = sal[i];
      for (int j : js) m = std::max(m, sal_in[j]);
      sal[i] = m;
      acc[i] += (i64)js.size();
      last[i] = now;
      ib[i] = imp_b(acc[i]);
      ic[i] = imp_c(now, now);
      seg->touched.insert(r);
    }
    return kept;
  }

  void insert(const std::vector<int>& kept) {
    for (int j : kept) {
      const i64 key = next_row++;
      fact_key[j] = key;
      key_fact[key] = j;
      fact_live[j] = 1;
      add_state(key, sal_in[j], code[j], false, fact_n2[j]);
      ++shard_count[code[j]];
      ++node_count;
      seg->inserts.push_back({0, j});
      ++stats["inserted"];
    }
  }

  void edge(i64 s, i64 d, float w, i64 h, int c) {
    const int e = (int)e_src.size();
    e_src.push_back(s);
    e_dst.push_back(d);
    e_code.push_back(h);
    e_conv.push_back(c);
    e_w.push_back(w);
    e_alive.push_back(1);
    inc[s].push_back(e);
    inc[d].push_back(e);
    seg->edges.push_back(e);
    ++stats["linked"];
  }

  void link(const std::vector<int>& kept, int c) {
    if (kept.empty()) return;
    const int k = (int)kept.size();
    std::vector<int> order(k);
    for (int i = 0; i < k; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return code[kept[a]] < code[kept[b]]; });
    for (int p = 0; p + 1 < k; ++p) {
      const int a = kept[order[p]], b = kept[order[p + 1]];
      if (code[a] == code[b]) edge(fact_key[a], fact_key[b], chain_w, code[a], c);
    }
    std::map<i64, int> cnt;
    for (int j : kept) ++cnt[code[j]];
    std::unordered_map<int, std::vector<i64>> within;
    std::vector<Cand> cl;
    for (int j : kept) {
      if (cnt[code[j]] < 2) continue;
      auto& w = within[j];
      cands(j, true, c, cl);
      for (int t = 0; t < (int)cl.size() && t < link_k; ++t) {
        edge(fact_key[j], cl[t].r, (float)(cl[t].v * link_scale), code[j], c);
        w.push_back(cl[t].r);
      }
    }
    for (int j : kept) {
      cands(j, false, c, cl);
      auto it = within.find(j);
      for (int t = 0; t < (int)cl.size() && t < link_k; ++t) {
        if (it != within.end() && std::find(it->second.begin(), it->second.end(), cl[t].r) != it->second.end())
          continue;
        edge(fact_key[j], cl[t].r, (float)(cl[t].v * link_scale), code[j], c);
        ++stats["cross_links"];
      }
    }
  }

  std::vector<double> imp_buf;
  std::vector<int> li;

  void evict(int c) {
    const i64 excess = node_count - max_buffer;
    if (excess <= 0) return;
    // the m = excess smallest (importance, shard, row) keys of the evictable
    // rows in ONE pass: a bounded max-heap (m is a handful of rows per
    // conversation, the pool thousands) instead of collecting every row and
    // nth_element -- the same rows in the same order (the key is a total order)
    if (imp_buf.size() < row.size()) imp_buf.resize(row.size());
    double* imp = imp_buf.data();
    auto less = [&](int a, int b) {
      if (imp[a] != imp[b]) return imp[a] < imp[b];
      if (ncode[a] != ncode[b]) return ncode[a] < ncode[b];
      return row[a] < row[b];
    };
    const size_t mx = (size_t)excess;
    li.clear();
    for (int i = 0; i < (int)row.size(); ++i) {
      if (!(cand[i] && alive[i])) continue;
      imp[i] = importance_bc(sal[i], ib[i], ic[i]);
      if (li.size() < mx) {
        li.push_back(i);
        std::push_heap(li.begin(), li.end(), less);
      } else if (less(i, li.front())) {
        std::pop_heap(li.begin(), li.end(), less);
        li.back() = i;
        std::push_heap(li.begin(), li.end(), less);
      }
    }
    if (li.empty()) return;
    std::sort_heap(li.begin(), li.end(), less);
    const size_t m = li.size();
    const int lastv = li[m - 1];
    events.emplace_back(decays, imp[lastv], ncode[lastv], row[lastv]);
    for (size_t t = 0; t < m; ++t) {
      const int i = li[t];
      const i64 r = row[i];
      alive[i] = 0;
      evicted[r] = c;
      if (r < n0) evicted_pre.push_back(r);
      auto kf = key_fact.find(r);
      if (kf != key_fact.end()) fact_live[kf->second] = 0;
      --node_count;
      --shard_count[ncode[i]];
      seg->victims.push_back(r);
      seg->touched.insert(r);
      ++stats["evicted"];
      auto ie = inc.find(r);
      if (ie != inc.end())
        for (int e : ie->second)
          if (e_alive[e] && e_code[e] == ncode[i]) e_alive[e] = 0;
    }
  }

  void make_supers(const std::vector<int>& kept, int c) {
    if (!ref_h) return;
    std::vector<i64> seen;
    for (int j : kept)
      if (std::find(seen.begin(), seen.end(), code[j]) == seen.end()) seen.push_back(code[j]);
    for (i64 cd : seen) {
      if ((double)shard_count[cd] <= sthr || (double)shard_count[cd] < sthr || super_codes.count(cd)) continue;
      const i64 key = next_row++;
      std::vector<i64> children;
      py::gil_scoped_acquire gil;  // (run() releases the GIL; the callbacks are Python)
      auto pre = py::cast<arr<i64>>(pre_members(cd));
      for (py::ssize_t t = 0; t < pre.size(); ++t)
        if (present(pre.data()[t])) children.push_back(pre.data()[t]);
      std::vector<i64> new_facts;
      for (int j = 0; j < M; ++j)
        if (fact_key[j] >= 0 && code[j] == cd && present(fact_key[j])) {
          children.push_back(fact_key[j]);
          new_facts.push_back(j);
        }
      py::tuple res = super_cos_fn(py::array_t<i64>(children.size(), children.data()),
                                   py::array_t<i64>(new_facts.size(), new_facts.data()));
      auto cs = py::cast<arr<double>>(res[0]);
      Super sp{cd, key, c, children, std::vector<double>(cs.data(), cs.data() + cs.size()),
               py::cast<double>(res[1])};
      if ((int)sp.cos.size() < M) sp.cos.resize(M, -INFINITY);
      supers.push_back(std::move(sp));
      super_codes.insert(cd);
      ++node_count;
      add_state(key, 0.5f, cd, true, supers.back().n2);
      seg->inserts.push_back({1, (int)supers.size() - 1});
    }
  }

  void end_decay() {
    ++decays;
    // branch-free over every row (the same rounding as decay_sal): live shard
    // nodes decay towards the floor, every other row keeps its salience
    const size_t R = row.size();
    float* sp = sal.data();
    const uint8_t* al = alive.data();
    const uint8_t* su = sup.data();
    for (size_t i = 0; i < R; ++i) {
      const float s = sp[i];
      const float d = s - kSalFloor;
      const float m = d * keep;
      const float v = s > kSalFloor ? kSalFloor + m : kSalFloor;
      sp[i] = (al[i] & (su[i] == 0)) ? v : s;
    }
    for (size_t e = 0; e < e_w.size(); ++e) {
      if (!e_alive[e]) continue;
      const float w = e_w[e] * keep;
      e_w[e] = w;
      if (has_thr && w < thr) {
        e_alive[e] = 0;
        ++stats["pruned_new"];
      }
    }
  }

  void close() {
    Seg& s = *seg;
    std::unordered_set<i64> new_keys;
    for (auto [kind, idx] : s.inserts) {
      const i64 key = kind == 0 ? fact_key[idx] : supers[idx].key;
      new_keys.insert(key);
      const int i = loc.at(key);
      s.ins_sal.push_back(sal[i]);
      s.ins_acc.push_back(acc[i]);
      s.ins_last.push_back(last[i]);
    }
    for (i64 r : s.touched) {
      if (new_keys.count(r)) continue;
      const int i = loc.at(r);
      s.tch_rows.push_back(r);
      s.tch_sal.push_back(sal[i]);
      s.tch_acc.push_back(acc[i]);
      s.tch_last.push_back(last[i]);
    }
    std::vector<int> live;
    for (int e : s.edges)
      if (e_alive[e]) {
        live.push_back(e);
        s.edge_w.push_back(e_w[e]);
      }
    s.edges.swap(live);
  }

  // seg_each: close a segment after EVERY conversation (a durable commit
  // per conversation, like the reference's save per end_conversation)
  double tprof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  void run(int B, i64 count0, bool autoc, i64 every, i64 cluster_every, bool seg_each) {
    next_row = n0;
    double t0 = now_s();
    build_near();
    tprof[0] += now_s() - t0;
    segs.clear();
    segs.push_back(Seg{0, 0});
    seg = &segs.back();
    int j0 = 0;
    for (int c = 0; c < B; ++c) {
      seg->c1 = c;
      conv_first = j0;
      std::vector<int> jj;
      while (j0 < M && ct[j0] == c) jj.push_back(j0++);
      double t1 = now_s();
      auto kept = dedupe(jj, c);
      double t2 = now_s();
      insert(kept);
      link(kept, c);
      double t3 = now_s();
      evict(c);
      make_supers(kept, c);
      double t4 = now_s();
      end_decay();
      double t5 = now_s();
      evict(c);
      double t6 = now_s();
      tprof[1] += t2 - t1; tprof[2] += t3 - t2; tprof[3] += t4 - t3 + t6 - t5; tprof[4] += t5 - t4;
      const i64 count = count0 + c + 1;
      const bool point = autoc && every > 0 && count % every == 0;
      const bool clus = cluster_every > 0 && count / cluster_every > (count - 1) / cluster_every;
      if (point || clus || seg_each || c == B - 1) {
        seg->consolidate = point;
        seg->cluster = clus;
        double t7 = now_s();
        close();
        tprof[5] += now_s() - t7;
        if (c < B - 1) {
          segs.push_back(Seg{c + 1, c + 1});
          seg = &segs.back();
        }
      }
    }
  }
};

template <class T>
std::vector<T> vec(py::handle h) {
  auto a = py::cast<arr<T>>(h);
  return std::vector<T>(a.data(), a.data() + a.size());
}

template <class T>
py::array_t<T> out(const std::vector<T>& v) {
  return py::array_t<T>(v.size(), v.data());
}

py::dict plan_batch(py::dict kw) {
  const double tin = Planner::now_s();
  Planner p;
  p.ct = vec<i64>(kw["ct"]);
  p.code = vec<i64>(kw["code"]);
  p.sal_in = vec<float>(kw["sal_in"]);
  p.M = (int)p.ct.size();
  p.n0 = py::cast<i64>(kw["n0"]);
  p.node_count = py::cast<i64>(kw["node_count"]);
  p.shard_count = vec<i64>(kw["shard_count"]);
  for (i64 c : vec<i64>(kw["super_codes"])) p.super_codes.insert(c);
  p.max_buffer = py::cast<i64>(kw["max_buffer"]);
  p.sthr = py::cast<double>(kw["super_threshold"]);
  p.ref_h = py::cast<bool>(kw["ref_hierarchy"]);
  p.has_thr = !kw["prune_thr"].is_none();
  p.thr = p.has_thr ? py::cast<float>(kw["prune_thr"]) : 0.f;
  p.keep = py::cast<float>(kw["keep"]);
  p.now = py::cast<double>(kw["now"]);
  p.gs = vec<double>(kw["gs"]);
  p.gr = vec<i64>(kw["gr"]);
  p.ss = vec<double>(kw["ss"]);
  p.sr = vec<i64>(kw["sr"]);
  p.K = p.M ? (int)(p.gs.size() / p.M) : 0;
  p.sup_rows = vec<i64>(kw["sup_rows"]);
  p.S = (int)p.sup_rows.size();
  p.sup_cos = vec<double>(kw["sup_cos"]);
  p.sup_n2 = vec<double>(kw["sup_n2"]);
  p.Sarr = py::cast<arr<double>>(kw["S"]);
  p.Sp = p.Sarr.data();
  p.qnorm = vec<double>(kw["qnorm"]);
  p.fact_n2 = vec<double>(kw["fact_n2"]);
  p.dedupe_thr = py::cast<double>(kw["dedupe_thr"]);
  p.link_thr = py::cast<double>(kw["link_thr"]);
  p.link_k = py::cast<int>(kw["link_k"]);
  p.link_scale = py::cast<double>(kw["link_scale"]);
  p.chain_w = py::cast<float>(kw["chain_w"]);
  p.pre_members = kw["pre_members"];
  p.super_cos_fn = kw["super_cos"];
  p.fallback_fn = kw["fallback"];
  {
    auto rows = vec<i64>(kw["rows"]);
    auto sal = vec<float>(kw["sal"]);
    auto acc = vec<i64>(kw["acc"]);
    auto last = vec<double>(kw["last"]);
    auto ncode = vec<i64>(kw["ncode"]);
    auto sup = vec<uint8_t>(kw["sup"]);
    auto n2 = vec<double>(kw["n2"]);
    auto pool = vec<uint8_t>(kw["pool"]);
    const size_t R = rows.size();
    if (sal.size() != R || acc.size() != R || last.size() != R || ncode.size() != R || sup.size() != R ||
        n2.size() != R || pool.size() != R)
      throw std::invalid_argument("plan_batch: row state columns differ in length");
    p.row = rows;
    p.sal = sal;
    p.acc = acc;
    p.last = last;
    p.ncode = ncode;
    p.sup = sup;
    p.n2 = n2;
    p.alive.assign(R, 1);
    p.cand.resize(R);
    p.ib.resize(R);
    p.ic.resize(R);
    for (size_t i = 0; i < R; ++i) {
      p.cand[i] = pool[i] && !sup[i];
      p.loc[rows[i]] = (int)i;
      p.ib[i] = imp_b(acc[i]);
      p.ic[i] = imp_c(last[i], p.now);
    }
  }
  const size_t M = p.M;
  if (p.sal_in.size() != M || p.code.size() != M || p.qnorm.size() != M || p.fact_n2.size() != M ||
      (size_t)p.Sarr.size() != M * M || p.gr.size() != p.gs.size() || p.ss.size() != p.gs.size() ||
      p.sr.size() != p.gs.size() || p.sup_cos.size() != M * (size_t)p.S || p.sup_n2.size() != (size_t)p.S)
    throw std::invalid_argument("plan_batch: inconsistent fact inputs");
  for (size_t j = 1; j < M; ++j)
    if (p.ct[j] < p.ct[j - 1]) throw std::invalid_argument("plan_batch: facts must be in conversation order");
  for (i64 c : p.code)
    if (c < 0 || c >= (i64)p.shard_count.size()) throw std::invalid_argument("plan_batch: shard code out of range");
  p.fact_key.assign(M, -1);
  p.dup_of.assign(M, -1);
  p.fact_live.assign(M, 0);
  const int a_B = py::cast<int>(kw["B"]);
  const i64 a_c0 = py::cast<i64>(kw["count0"]), a_every = py::cast<i64>(kw["every"]),
            a_cl = py::cast<i64>(kw["cluster_every"]);
  const bool a_auto = py::cast<bool>(kw["auto"]), a_seg = kw.contains("seg_each") && py::cast<bool>(kw["seg_each"]);
  const double trun = Planner::now_s();
  {
    // the plan itself is pure C++ over copied / held arrays: other Python
    // threads (a write-behind persistence, a serving loop) run meanwhile
    py::gil_scoped_release nogil;
    p.run(a_B, a_c0, a_auto, a_every, a_cl, a_seg);
  }
  const double tout = Planner::now_s();

  py::list segs;
  for (auto& s : p.segs) {
    py::dict d;
    std::vector<int> kinds, idx;
    for (auto [k, i] : s.inserts) {
      kinds.push_back(k);
      idx.push_back(i);
    }
    std::vector<i64> es, ed, ec;
    for (int e : s.edges) {
      es.push_back(p.e_src[e]);
      ed.push_back(p.e_dst[e]);
      ec.push_back(p.e_code[e]);
    }
    d["c0"] = s.c0;
    d["c1"] = s.c1;
    d["consolidate"] = s.consolidate;
    d["cluster"] = s.cluster;
    d["ins_kind"] = out(kinds);
    d["ins_idx"] = out(idx);
    d["ins_sal"] = out(s.ins_sal);
    d["ins_acc"] = out(s.ins_acc);
    d["ins_last"] = out(s.ins_last);
    d["edge_src"] = out(es);
    d["edge_dst"] = out(ed);
    d["edge_code"] = out(ec);
    d["edge_w"] = out(s.edge_w);
    d["victims"] = out(s.victims);
    d["tch_rows"] = out(s.tch_rows);
    d["tch_sal"] = out(s.tch_sal);
    d["tch_acc"] = out(s.tch_acc);
    d["tch_last"] = out(s.tch_last);
    segs.append(d);
  }
  py::list sups;
  for (auto& sp : p.supers) {
    py::dict d;
    d["code"] = sp.code;
    d["key"] = sp.key;
    d["conv"] = sp.conv;
    d["children"] = out(sp.children);
    sups.append(d);
  }
  py::list ev;
  for (auto& [st, imp, cd, r] : p.events) ev.append(py::make_tuple(st, imp, cd, r));
  py::dict res;
  res["segments"] = segs;
  res["supers"] = sups;
  res["events"] = ev;
  res["fact_key"] = out(p.fact_key);
  res["dup_of"] = out(p.dup_of);
  py::dict st;
  for (auto& [k, v] : p.stats) st[py::str(k)] = v;
  res["stats"] = st;
  if (std::getenv("LZK_PLAN_PROF"))  // diagnostic: planner phases (tools/plan_bench.py)
    std::fprintf(stderr,
                 "plan_batch ms: inputs %.3f near %.3f dedupe %.3f insert+link %.3f evict+supers %.3f "
                 "decay %.3f close %.3f outputs %.3f\n",
                 (trun - tin) * 1e3, p.tprof[0] * 1e3, p.tprof[1] * 1e3, p.tprof[2] * 1e3, p.tprof[3] * 1e3,
                 p.tprof[4] * 1e3, p.tprof[5] * 1e3, (Planner::now_s() - tout) * 1e3);
  return res;
}

}  // namespace

namespace lzrt {
void register_batch_plan(py::module_& m) {
  m.def("plan_batch", &plan_batch, py::arg("kw"),
        "Plan B sequential end_conversation calls (MemorySystem.consolidate_batch); see core/batch_plan.py");
}
}  // namespace lzrt
