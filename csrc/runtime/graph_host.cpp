#include "graph_host.h"

#include <numeric>

namespace lzrt {

void build_csr(const int32_t* src, const int32_t* dst, int64_t ne, int n, bool undirected,
               std::vector<int64_t>& off, std::vector<int32_t>& adj, std::vector<int32_t>& eid) {
  off.assign((size_t)n + 1, 0);
  for (int64_t e = 0; e < ne; ++e) {
    off[src[e] + 1]++;
    if (undirected && src[e] != dst[e]) off[dst[e] + 1]++;
  }
  for (int i = 0; i < n; ++i) off[i + 1] += off[i];
  adj.assign(off[n], 0);
  eid.assign(off[n], 0);
  std::vector<int64_t> cur(off.begin(), off.end() - 1);
  for (int64_t e = 0; e < ne; ++e) {
    int64_t p = cur[src[e]]++;
    adj[p] = dst[e];
    eid[p] = (int32_t)e;
    if (undirected && src[e] != dst[e]) {
      p = cur[dst[e]]++;
      adj[p] = src[e];
      eid[p] = (int32_t)e;
    }
  }
}

static int32_t find(std::vector<int32_t>& p, int32_t x) {
  while (p[x] != x) { p[x] = p[p[x]]; x = p[x]; }
  return x;
}

void union_find(const int32_t* src, const int32_t* dst, int64_t ne, int n, std::vector<int32_t>& label) {
  label.resize(n);
  std::iota(label.begin(), label.end(), 0);
  for (int64_t e = 0; e < ne; ++e) {
    int32_t a = find(label, src[e]), b = find(label, dst[e]);
    if (a == b) continue;
    if (a < b) label[b] = a; else label[a] = b;  // min-label root
  }
  for (int i = 0; i < n; ++i) label[i] = find(label, i);
}

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

static uint64_t tenant_hash(const std::string& tenant) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : tenant) { h ^= c; h *= 1099511628211ull; }
  return h;
}

int tenant_rank(const std::string& tenant, int world) {
  // rendezvous (highest-random-weight) hashing: adding a rank moves only
  // the tenants that now score highest on it.
  const uint64_t h = tenant_hash(tenant);
  int best = 0;
  uint64_t bw = 0;
  for (int r = 0; r < world; ++r) {
    uint64_t w = mix64(h ^ (0x9e3779b97f4a7c15ull * (uint64_t)(r + 1)));
    if (r == 0 || w > bw) { bw = w; best = r; }
  }
  return best;
}

int tenant_rank_among(const std::string& tenant, const std::vector<int>& ranks) {
  // same weights as tenant_rank restricted to the surviving rank ids: when a
  // rank leaves, only the tenants it owned move (each to its runner-up).
  const uint64_t h = tenant_hash(tenant);
  int best = -1;
  uint64_t bw = 0;
  for (int r : ranks) {
    uint64_t w = mix64(h ^ (0x9e3779b97f4a7c15ull * (uint64_t)(r + 1)));
    if (best < 0 || w > bw) { bw = w; best = r; }
  }
  return best;
}

}  // namespace lzrt
