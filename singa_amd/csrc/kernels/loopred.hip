// Device reduction of the loopback world's CAPTURED all-reduce
// (csrc/comm/loop_comm.cpp): when every rank thread of an in-process world
// captures its step into ONE HIP graph, a collective becomes graph edges
// (each rank's stream -> this kernel -> each rank's stream) plus this kernel,
// which reads every rank's send buffer and writes every rank's receive
// buffer.  Element i is read from all ranks and written to all ranks by the
// same lane, so in-place calls (send == recv, DistOpt's buckets) are safe.
// Rank order and fp32 accumulation as the host path (deterministic).
#include "common.h"

namespace {
constexpr int kMaxRanks = 16;
struct Ptrs {
  const void* send[kMaxRanks];
  void* recv[kMaxRanks];
};

// op: 0 sum, 2 max, 3 min, 4 avg
template <typename T, typename A>
__global__ void __launch_bounds__(256) loop_allreduce_k(Ptrs p, int n, int64_t count, int op) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
    A acc = (A)((const T*)p.send[0])[i];
    for (int r = 1; r < n; ++r) {
      const A v = (A)((const T*)p.send[r])[i];
      acc = op == 2 ? (v > acc ? v : acc) : op == 3 ? (v < acc ? v : acc) : acc + v;
    }
    if (op == 4) acc = acc / (A)n;
    const T out = (T)acc;
    for (int r = 0; r < n; ++r) ((T*)p.recv[r])[i] = out;
  }
}
}  // namespace

extern "C" int sg_loop_allreduce(const void* const* sends, void* const* recvs, int n, int64_t count, int dt, int op,
                                 hipStream_t s) {
  if (n < 1 || n > kMaxRanks || count < 0) return -1;
  if (count == 0) return 0;
  Ptrs p;
  for (int r = 0; r < n; ++r) {
    p.send[r] = sends[r];
    p.recv[r] = recvs[r];
  }
  const int blocks = (int)((count + 255) / 256 < 4096 ? (count + 255) / 256 : 4096);
  switch (dt) {
    case 0: hipLaunchKernelGGL((loop_allreduce_k<float, float>), dim3(blocks), dim3(256), 0, s, p, n, count, op); break;
    case 1: hipLaunchKernelGGL((loop_allreduce_k<sg::bf16, float>), dim3(blocks), dim3(256), 0, s, p, n, count, op); break;
    case 6: hipLaunchKernelGGL((loop_allreduce_k<double, double>), dim3(blocks), dim3(256), 0, s, p, n, count, op); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
