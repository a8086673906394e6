// Host graph utilities: CSR build (counting sort), union-find components and
// rendezvous-hash tenant placement. Device-scale equivalents are HIP kernels
// (csrc/kernels/graph.hip); these serve the host paths and test oracles.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace lzrt {
void build_csr(const int32_t* src, const int32_t* dst, int64_t ne, int n, bool undirected,
               std::vector<int64_t>& off, std::vector<int32_t>& adj, std::vector<int32_t>& eid);
void union_find(const int32_t* src, const int32_t* dst, int64_t ne, int n, std::vector<int32_t>& label);
int tenant_rank(const std::string& tenant, int world);
int tenant_rank_among(const std::string& tenant, const std::vector<int>& ranks);
}  // namespace lzrt
