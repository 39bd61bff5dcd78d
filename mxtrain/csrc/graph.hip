// hipGraph post-processing between capture and instantiation (host code, HIP runtime API).
//
// Why: with the HIP runtime's graph packet capture (dispatch packets pre-built at
// instantiation, DEBUG_CLR_GRAPH_PACKET_CAPTURE=1, the runtime default), a captured
// host-to-device memcpy node breaks the ordering of later memset nodes against the kernels
// around them: scripts/probe_graph_nodes.py, one MI355X, ROCm 7 runtime -- a graph of
// [H2D copy] then 50 x [memset acc, add_one, add_one, snapshot] replays with one round's
// snapshot wrong, while the same graph without the H2D node, or with packet capture off,
// replays exactly.  The whole-step Mask R-CNN graph holds such nodes (library code stages
// arguments host -> device inside the capture) and its memsets zero buffers that are then
// accumulated into and used for indexing, hence the illegal-address fault of the replay.
//
// Fix: after capture, every memcpy node whose source is host memory is rewritten into a
// device-to-device copy from a device snapshot of the source bytes taken at rewrite time.
// That is also the only meaning such a node can have in a replayed graph (CUDA refuses a
// pageable-source copy during capture outright; HIP records it and re-reads the host
// buffer at every replay -- by then usually freed and reused, see the probe).  The snapshots
// live as long as the graph (the caller frees them with mx_graph_free).
#include "common.h"

#include <vector>

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

namespace {

// Parameters of a memcpy node through the driver-style getter (HIP_MEMCPY3D: memory types,
// host / device pointers, widths), which this runtime fills for the 1-D copies stream
// capture records; hipGraphMemcpyNodeGetParams leaves its hipMemcpy3DParms unfilled for
// them (scripts/probe_graph_nodes.py).  Returns false when the node cannot be read or is
// not a plain 1-D linear copy.
struct Copy1D {
  const void* src;
  void* dst;
  size_t bytes;
  bool src_host, dst_host;
};
bool read_copy(hipGraphNode_t nd, Copy1D& c) {
  HIP_MEMCPY3D p{};
  if (hipDrvGraphMemcpyNodeGetParams(nd, &p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (p.srcArray || p.dstArray || p.Height > 1 || p.Depth > 1 || p.srcY || p.srcZ || p.dstY || p.dstZ)
    return false;
  c.src_host = p.srcMemoryType == hipMemoryTypeHost || p.srcMemoryType == hipMemoryTypeUnregistered;
  c.dst_host = p.dstMemoryType == hipMemoryTypeHost || p.dstMemoryType == hipMemoryTypeUnregistered;
  c.src = c.src_host ? (const char*)p.srcHost + p.srcXInBytes : (const char*)p.srcDevice + p.srcXInBytes;
  c.dst = c.dst_host ? (char*)p.dstHost + p.dstXInBytes : (char*)p.dstDevice + p.dstXInBytes;
  c.bytes = p.WidthInBytes;
  return true;
}

}  // namespace

// rows of {src, dst, bytes, src_memory_type, dst_memory_type} for every memcpy node (up to
// max_rows; memory type 1 = host, 2 = device, -1 = unreadable node); returns the number of
// memcpy nodes or -1 on an API error
MX_EXPORT int mx_graph_memcpy_nodes(void* graph, int64_t* out, int max_rows) {
  std::vector<hipGraphNode_t> nodes;
  if (graph_nodes((hipGraph_t)graph, nodes) < 0) return -1;
  int k = 0;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nd, &t) != hipSuccess) return -1;
    if (t != hipGraphNodeTypeMemcpy) continue;
    if (k < max_rows) {
      int64_t* r = out + 5 * k;
      Copy1D c{};
      if (read_copy(nd, c)) {
        r[0] = (int64_t)(uintptr_t)c.src;
        r[1] = (int64_t)(uintptr_t)c.dst;
        r[2] = (int64_t)c.bytes;
        r[3] = c.src_host ? 1 : 2;
        r[4] = c.dst_host ? 1 : 2;
      } else {
        r[0] = r[1] = r[2] = 0;
        r[3] = r[4] = -1;
      }
    }
    ++k;
  }
  return k;
}

// Rewrite host-to-device 1-D memcpy nodes into device-to-device copies from device
// snapshots (see the top of the file).  snaps receives the device buffers (at most
// max_snaps); returns the number of rewritten nodes, or a negative error without having
// changed anything (-1 API, -2 a memcpy node is unreadable, -5 too many), or -4 after an
// allocation failure.
MX_EXPORT int mx_graph_snapshot_h2d(void* graph, void** snaps, int max_snaps) {
  std::vector<hipGraphNode_t> nodes;
  if (graph_nodes((hipGraph_t)graph, nodes) < 0) return -1;
  std::vector<std::pair<hipGraphNode_t, Copy1D>> todo;
  for (auto nd : nodes) {   // read everything first: all-or-nothing
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nd, &t) != hipSuccess) return -1;
    if (t != hipGraphNodeTypeMemcpy) continue;
    Copy1D c{};
    if (!read_copy(nd, c)) return -2;
    if (c.src_host && !c.dst_host) todo.emplace_back(nd, c);
  }
  if ((int)todo.size() > max_snaps) return -5;
  int k = 0;
  for (auto& [nd, c] : todo) {
    void* d = nullptr;
    if (hipMalloc(&d, c.bytes ? c.bytes : 1) != hipSuccess) return -4;
    if (c.bytes && hipMemcpy(d, c.src, c.bytes, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(d);
      return -1;
    }
    if (hipGraphMemcpyNodeSetParams1D(nd, c.dst, d, c.bytes, hipMemcpyDeviceToDevice) != hipSuccess) {
      (void)hipFree(d);
      return -1;
    }
    snaps[k++] = d;
  }
  return k;
}

MX_EXPORT int mx_graph_free(void** bufs, int n) {
  for (int i = 0; i < n; ++i)
    if (bufs[i]) (void)hipFree(bufs[i]);
  return 0;
}
