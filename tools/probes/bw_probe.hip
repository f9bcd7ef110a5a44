// Streaming-bandwidth probe for the BN apply passes: which access pattern
// gets closest to HBM3E peak on MI355X for a read-x/write-y elementwise pass
// over a ~1.6 GB bf16 tensor.  Build: hipcc -O3 --offload-arch=gfx950 bw_probe.hip -o bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// grid-stride, UR 16-byte loads in flight per thread, optional nontemporal
template <int UR, bool NT>
__global__ void __launch_bounds__(256) copy_k(const u32x4* __restrict__ x, u32x4* __restrict__ y, long n) {
  const long step = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UR - 1) * step < n; i += UR * step) {
    u32x4 v[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) v[u] = NT ? __builtin_nontemporal_load(x + i + u * step) : x[i + u * step];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], y + i + u * step);
      else y[i + u * step] = v[u];
    }
  }
  for (; i < n; i += step) y[i] = x[i];
}

// contiguous chunk per workgroup: each WG streams CH consecutive 4 KB blocks
template <int UR, bool NT>
__global__ void __launch_bounds__(256) chunk_k(const u32x4* __restrict__ x, u32x4* __restrict__ y, long n, long per_wg) {
  long b = (long)blockIdx.x * per_wg;
  long e = b + per_wg < n ? b + per_wg : n;
  for (long i = b + threadIdx.x; i < e; i += 256 * UR) {
    u32x4 v[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const long j = i + u * 256;
      if (j < e) v[u] = NT ? __builtin_nontemporal_load(x + j) : x[j];
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const long j = i + u * 256;
      if (j < e) {
        if (NT) __builtin_nontemporal_store(v[u], y + j);
        else y[j] = v[u];
      }
    }
  }
}

// one block of 256*UR vectors per workgroup, no loop (huge grid)
template <int UR, bool NT>
__global__ void __launch_bounds__(256) oneshot_k(const u32x4* __restrict__ x, u32x4* __restrict__ y, long n) {
  const long b = (long)blockIdx.x * 256 * UR + threadIdx.x;
  u32x4 v[UR];
#pragma unroll
  for (int u = 0; u < UR; ++u)
    if (b + u * 256 < n) v[u] = NT ? __builtin_nontemporal_load(x + b + u * 256) : x[b + u * 256];
#pragma unroll
  for (int u = 0; u < UR; ++u)
    if (b + u * 256 < n) {
      if (NT) __builtin_nontemporal_store(v[u], y + b + u * 256);
      else y[b + u * 256] = v[u];
    }
}

int main() {
  const long bytes = 1644167168L;  // 1024 x 56 x 56 x 256 bf16
  const long n = bytes / 16;
  u32x4 *x, *y;
  hipMalloc(&x, bytes);
  hipMalloc(&y, bytes);
  hipMemset(x, 1, bytes);
  hipMemset(y, 0, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(a);
    const int it = 10;
    for (int k = 0; k < it; ++k) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= it;
    printf("{\"variant\": \"%s\", \"us\": %.1f, \"GBps\": %.0f}\n", name, ms * 1e3, 2.0 * bytes / (ms * 1e-3) / 1e9);
  };
  for (int rep = 0; rep < 2; ++rep) {
    run("gs_ur1_g1024", [&] { hipLaunchKernelGGL((copy_k<1, false>), dim3(1024), dim3(256), 0, 0, x, y, n); });
    run("gs_ur1_nt_g1024", [&] { hipLaunchKernelGGL((copy_k<1, true>), dim3(1024), dim3(256), 0, 0, x, y, n); });
    run("gs_ur1_g512", [&] { hipLaunchKernelGGL((copy_k<1, false>), dim3(512), dim3(256), 0, 0, x, y, n); });
    for (int g : {32768, 65536, 131072}) {
      const long per = (n + g - 1) / g;
      char nm[64];
      snprintf(nm, 64, "chunk_ur4_nt_g%d", g);
      run(nm, [&] { hipLaunchKernelGGL((chunk_k<4, true>), dim3(g), dim3(256), 0, 0, x, y, n, per); });
      snprintf(nm, 64, "chunk_ur2_nt_g%d", g);
      run(nm, [&] { hipLaunchKernelGGL((chunk_k<2, true>), dim3(g), dim3(256), 0, 0, x, y, n, per); });
      snprintf(nm, 64, "chunk_ur4_g%d", g);
      run(nm, [&] { hipLaunchKernelGGL((chunk_k<4, false>), dim3(g), dim3(256), 0, 0, x, y, n, per); });
    }
    run("oneshot_ur1", [&] { hipLaunchKernelGGL((oneshot_k<1, false>), dim3((n + 255) / 256), dim3(256), 0, 0, x, y, n); });
    run("oneshot_ur1_nt", [&] { hipLaunchKernelGGL((oneshot_k<1, true>), dim3((n + 255) / 256), dim3(256), 0, 0, x, y, n); });
    run("oneshot_ur2_nt", [&] { hipLaunchKernelGGL((oneshot_k<2, true>), dim3((n + 511) / 512), dim3(256), 0, 0, x, y, n); });
    run("oneshot_ur4", [&] { hipLaunchKernelGGL((oneshot_k<4, false>), dim3((n + 1023) / 1024), dim3(256), 0, 0, x, y, n); });
    run("oneshot_ur4_nt", [&] { hipLaunchKernelGGL((oneshot_k<4, true>), dim3((n + 1023) / 1024), dim3(256), 0, 0, x, y, n); });
  }
  run("hipMemcpyDtoD", [&] { hipMemcpyAsync(y, x, bytes, hipMemcpyDeviceToDevice, 0); });
  return 0;
}
