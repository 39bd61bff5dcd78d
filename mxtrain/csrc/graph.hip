// hipGraph post-processing between capture and instantiation (HIP runtime API + one fill
// kernel).
//
// Why: with the HIP runtime's graph packet capture (dispatch packets pre-built at
// instantiation, DEBUG_CLR_GRAPH_PACKET_CAPTURE, the runtime default), MEMSET NODES replay
// wrong on this runtime (one MI355X, profiles/r3_s4/):
//   * scripts/probe_graph_memsets.py: [copy, fill, memset, add, checksum] x 40 cases --
//     the first replay is exact, later replays get 4- and 12-byte memsets wrong;
//   * tests/test_graph_gpu.py: 64 x [16 KiB memset, add, add, D2D copy, add, snapshot] --
//     rounds wrong from the first replay;
//   * scripts/probe_graph_nodes.py: with a host-to-device copy node in front, the first
//     [memset, add, add, snapshot] round replays with garbage.
// With packet capture off every case is exact.  The Mask R-CNN whole-step graph holds 124
// memset nodes (MIOpen zeroes accumulation workspaces and index buffers with
// hipMemsetAsync), which is what made its replay take an illegal-address fault after a few
// steps with packet capture on.
//
// Fix: mx_graph_memsets_to_kernels replaces every memset node by a kernel node of
// graph_fill_kernel with the same parameters and the same dependency edges, so the graph
// holds only kernel (and copy) nodes and the packet-capture path builds ordinary dispatch
// packets for all of it.  mx_graph_census reports node kinds before / after.
#include "common.h"

#include <algorithm>
#include <vector>

namespace {

// memset semantics for a [height][width] region of elementSize-byte elements at `pitch`
// bytes per row: every element = value (1, 2 or 4 bytes).  Rows are filled in 16-byte
// vectors between an unaligned head and tail (the element pattern repeats every 16 bytes
// because elementSize divides 16 and dst is elementSize-aligned).
__global__ __launch_bounds__(256) void graph_fill_kernel(char* __restrict__ dst, size_t pitch, uint32_t value,
                                                         int esz, size_t width, size_t height) {
  const uint32_t v = esz == 1 ? (value & 0xFFu) * 0x01010101u : esz == 2 ? (value & 0xFFFFu) * 0x00010001u : value;
  const uint4 v4 = make_uint4(v, v, v, v);
  const size_t rowb = width * (size_t)esz;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
  for (size_t r = 0; r < height; ++r) {
    char* row = dst + r * pitch;
    const size_t head = min(rowb, (size_t)((16 - ((uintptr_t)row & 15)) & 15));
    const size_t nvec = (rowb - head) / 16;
    const size_t tail0 = head + nvec * 16;
    for (size_t i = tid; i < nvec; i += nth) *reinterpret_cast<uint4*>(row + head + 16 * i) = v4;
    for (size_t b = tid; b < head; b += nth) row[b] = (char)(v >> (8 * (((uintptr_t)row + b) & 3)));
    for (size_t b = tail0 + tid; b < rowb; b += nth) row[b] = (char)(v >> (8 * (((uintptr_t)row + b) & 3)));
  }
}

}  // namespace

namespace {

int graph_nodes(hipGraph_t g, std::vector<hipGraphNode_t>& nodes) {
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return -1;
  nodes.resize(n);
  if (n && hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return -1;
  nodes.resize(n);
  return (int)n;
}

}  // namespace

// counts[t] = number of nodes of hipGraphNodeType t (t < ncounts); returns the node count
MX_EXPORT int mx_graph_census(void* graph, int* counts, int ncounts) {
  std::vector<hipGraphNode_t> nodes;
  const int n = graph_nodes((hipGraph_t)graph, nodes);
  if (n < 0) return -1;
  for (int i = 0; i < ncounts; ++i) counts[i] = 0;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nd, &t) != hipSuccess) return -1;
    if ((int)t >= 0 && (int)t < ncounts) counts[(int)t]++;
  }
  return n;
}

// Replace every memset node of `graph` by a graph_fill_kernel node with the same region and
// value and the same incoming / outgoing edges (see the top of the file).  Returns the
// number of replaced nodes, or a negative error: -1 API failure, -2 a memset node whose
// parameters cannot be read (nothing is changed then), -3 an element size other than
// 1 / 2 / 4.
MX_EXPORT int mx_graph_memsets_to_kernels(void* graph) {
  hipGraph_t g = (hipGraph_t)graph;
  std::vector<hipGraphNode_t> nodes;
  if (graph_nodes(g, nodes) < 0) return -1;
  std::vector<std::pair<hipGraphNode_t, hipMemsetParams>> todo;
  for (auto nd : nodes) {   // read everything first: all-or-nothing
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nd, &t) != hipSuccess) return -1;
    if (t != hipGraphNodeTypeMemset) continue;
    hipMemsetParams p{};
    if (hipGraphMemsetNodeGetParams(nd, &p) != hipSuccess) {
      (void)hipGetLastError();
      return -2;
    }
    if (p.elementSize != 1 && p.elementSize != 2 && p.elementSize != 4) return -3;
    if (p.height == 0) p.height = 1;
    if (p.height > 1 && p.pitch < p.width * p.elementSize) return -2;
    todo.emplace_back(nd, p);
  }
  int k = 0;
  for (auto& [nd, p] : todo) {
    size_t nd_in = 0, nd_out = 0;
    if (hipGraphNodeGetDependencies(nd, nullptr, &nd_in) != hipSuccess) return -1;
    if (hipGraphNodeGetDependentNodes(nd, nullptr, &nd_out) != hipSuccess) return -1;
    std::vector<hipGraphNode_t> in(nd_in), out(nd_out);
    if (nd_in && hipGraphNodeGetDependencies(nd, in.data(), &nd_in) != hipSuccess) return -1;
    if (nd_out && hipGraphNodeGetDependentNodes(nd, out.data(), &nd_out) != hipSuccess) return -1;
    char* dst = (char*)p.dst;
    size_t pitch = p.height > 1 ? p.pitch : 0;
    uint32_t value = p.value;
    int esz = (int)p.elementSize;
    size_t width = p.width, height = p.height;
    const size_t bytes = width * (size_t)esz;
    const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>((bytes / 16 + 255) / 256, 1024));
    void* args[] = {&dst, &pitch, &value, &esz, &width, &height};
    hipKernelNodeParams kp{};
    kp.func = (void*)graph_fill_kernel;
    kp.gridDim = dim3(blocks);
    kp.blockDim = dim3(256);
    kp.kernelParams = args;
    kp.sharedMemBytes = 0;
    kp.extra = nullptr;
    hipGraphNode_t kn;
    if (hipGraphAddKernelNode(&kn, g, in.data(), in.size(), &kp) != hipSuccess) return -1;
    for (auto d : out)
      if (hipGraphAddDependencies(g, &kn, &d, 1) != hipSuccess) return -1;
    if (hipGraphDestroyNode(nd) != hipSuccess) return -1;
    ++k;
  }
  return k;
}
