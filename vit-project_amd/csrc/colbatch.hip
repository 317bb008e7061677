// Batched column reductions: every bias / LayerNorm-affine gradient of one transformer block's
// backward (qkv.bias, proj.bias, fc1.bias, fc2.bias, norm1/norm2 weight and
// bias) as ONE launch on the side stream, instead of one or two launches per gradient.
//
// A job is out[N] (+)= sum_r part[r][N] over the S partial rows a producing kernel wrote (the
// GEMM epilogues' 64-row column sums, the LayerNorm backward's per-block partials, the attention
// backward's per-image sums, the weight gradients' split-K slabs).
//   * short jobs (S <= 8: the split-K slabs of the weight-gradient pairs, 2..7 over ~2.4 M columns): a workgroup
//     takes 2048 columns, each lane 2 x 4 of them, and adds the S rows in row order (the order of
//     the former separate slab-reduce kernel, so the weight gradients are bit-identical to it);
//   * tall jobs (S > 8): workgroup = 64 partial rows x 256 columns (4 waves x 16 rows, one f32x4
//     per lane per row, all 16 loads in flight at once); a job with more than 64 rows has several
//     such chunks per 256-column strip: each chunk publishes its partial strip (agent-scope
//     release, then a ticket on the strip's counter) and the workgroup that draws the last ticket
//     sums the chunk partials in chunk order (MI355X_MICROARCH.md / cdna_hip_programming.md §5
//     "In-launch split-K reduction").
// Every sum runs in a fixed order, so the result does not depend on which workgroup finishes
// last.  Counters start at zero (zero-filled when the caller allocates them) and the last
// workgroup of each strip resets its counter.
#include "common.hpp"
#include "reduce.hpp"

namespace {
constexpr int CB_MAXJ = 16, CB_ROWS = 64, CB_COLS = 256;
constexpr int CB_SHORT = 8, CB_SHORT_COLS = 2048;  // short jobs: rows, columns per workgroup
struct CbJob {
  const float* part;
  float* out;
  int S, N, accumulate, strips, chunks, wg0, cnt0, pad;
  int64_t scr0;
};
struct CbJobs {
  CbJob j[CB_MAXJ];
  int n;
};

__device__ __forceinline__ void store_out(float* o, int col, int N, f32x4 v, int accumulate) {
  if (col + 4 <= N && ((uintptr_t)(o + col) & 15) == 0) {  // 16-B store (every output of the model)
    f32x4* p = reinterpret_cast<f32x4*>(o + col);
    *p = accumulate ? *p + v : v;
    return;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (col + t < N) o[col + t] = accumulate ? o[col + t] + v[t] : v[t];
}

__global__ __launch_bounds__(256) void colreduce_batch_kernel(CbJobs jobs, float* __restrict__ scratch,
                                                              int* __restrict__ cnt) {
  __shared__ f32x4 red[4][64];
  __shared__ int last;
  const int bid = blockIdx.x;
  int k = 0;
  while (k + 1 < jobs.n && bid >= jobs.j[k + 1].wg0) ++k;
  const CbJob& J = jobs.j[k];
  const int local = bid - J.wg0;
  if (J.S <= CB_SHORT) {  // rows added in row order, 2 x 4 columns per lane, all loads in flight
    f32x4 a[2], v[2][CB_SHORT];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = local * CB_SHORT_COLS + (u * 256 + threadIdx.x) * 4;
#pragma unroll
      for (int r = 0; r < CB_SHORT; ++r)
        if (r < J.S && c < J.N) v[u][r] = *reinterpret_cast<const f32x4*>(J.part + (int64_t)r * J.N + c);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = local * CB_SHORT_COLS + (u * 256 + threadIdx.x) * 4;
      if (c < J.N) {
        a[u] = v[u][0];
#pragma unroll
        for (int r = 1; r < CB_SHORT; ++r)
          if (r < J.S) a[u] += v[u][r];
        store_out(J.out, c, J.N, a[u], J.accumulate);
      }
    }
    return;
  }
  const int strip = local / J.chunks, chunk = local - strip * J.chunks;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = strip * CB_COLS + lane * 4;
  const bool cok = c < J.N;
  const int r0 = chunk * CB_ROWS;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (cok) {
    f32x4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = r0 + w + 4 * i;
      v[i] = r < J.S ? *reinterpret_cast<const f32x4*>(J.part + (int64_t)r * J.N + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) s += v[i];
  }
  red[w][lane] = s;
  __syncthreads();
  const f32x4 t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  if (J.chunks == 1) {
    if (w == 0 && cok) store_out(J.out, c, J.N, t, J.accumulate);
    return;
  }
  // publish this chunk's partial strip, then take a ticket on the strip's counter
  float* mine = scratch + J.scr0 + (int64_t)chunk * J.N;
  if (w == 0 && cok) *reinterpret_cast<f32x4*>(mine + c) = t;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tk = __hip_atomic_fetch_add(cnt + J.cnt0 + strip, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = tk == J.chunks - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(cnt + J.cnt0 + strip, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  // the chunk partials in chunk order, 4 columns per lane of wave 0 (the other waves idle)
  if (w == 0 && cok) {
    // eight loads in flight per step (a dependent load per chunk would pay the L2 latency 25 times);
    // the adds stay in chunk order
    const float* base = scratch + J.scr0 + c;
    f32x4 a = *reinterpret_cast<const f32x4*>(base);
    int q = 1;
    for (; q + 8 <= J.chunks; q += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4*>(base + (int64_t)(q + u) * J.N);
#pragma unroll
      for (int u = 0; u < 8; ++u) a += v[u];
    }
    for (; q < J.chunks; ++q) a += *reinterpret_cast<const f32x4*>(base + (int64_t)q * J.N);
    store_out(J.out, c, J.N, a, J.accumulate);
  }
}

bool job_vec_ok(const float* part, int N) { return N % 4 == 0 && ((uintptr_t)part & 15) == 0; }
}  // namespace

extern "C" {

// jobs: njobs x {part, out, S, N, accumulate} as int64 (host memory).  Scratch floats and
// counters the batch needs (jobs whose partials take the vector path and span > 64 rows).
int vit_colreduce_batch_sizes(const int64_t* jobs, int njobs, int64_t* scratch_floats, int* counters) {
  int64_t sf = 0;
  int nc = 0;
  for (int i = 0; i < njobs; ++i) {
    const int64_t* q = jobs + 5 * i;
    const int S = (int)q[2], N = (int)q[3];
    if (S <= 0 || N <= 0) continue;
    if (job_vec_ok((const float*)q[0], N)) {
      const int chunks = S <= CB_SHORT ? 1 : (S + CB_ROWS - 1) / CB_ROWS;
      if (chunks > 1) {
        sf += (int64_t)chunks * N;
        nc += (N + CB_COLS - 1) / CB_COLS;
      }
    } else {
      sf += colreduce_scratch_floats(S, N);
    }
  }
  *scratch_floats = sf;
  *counters = nc;
  return 0;
}

// out_i[N_i] (+)= sum over the S_i rows of part_i, for every job, in one launch (16 jobs per
// launch; jobs whose partials are not 16-B vectors take the two-stage colreduce).  scratch /
// counters as vit_colreduce_batch_sizes says; counters zero-filled before the first call (the
// kernel leaves them zero).
int vit_colreduce_batch(const int64_t* jobs, int njobs, float* scratch, int64_t scratch_floats, int* counters,
                        int ncounters, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int64_t need_sf = 0;
  int need_c = 0;
  vit_colreduce_batch_sizes(jobs, njobs, &need_sf, &need_c);
  if (scratch_floats < need_sf || ncounters < need_c || (need_c && !counters) || (need_sf && !scratch))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)scratch & 15) != 0) return (int)hipErrorInvalidValue;
  CbJobs b{};
  int wg = 0, cnt0 = 0;
  int64_t scr = 0;
  auto flush = [&]() {
    if (b.n == 0) return;
    hipLaunchKernelGGL(colreduce_batch_kernel, dim3(wg), dim3(256), 0, s, b, scratch, counters);
    b.n = 0;
    wg = 0;
  };
  for (int i = 0; i < njobs; ++i) {
    const int64_t* q = jobs + 5 * i;
    const float* part = (const float*)q[0];
    float* out = (float*)q[1];
    const int S = (int)q[2], N = (int)q[3], acc = (int)q[4];
    if (S <= 0 || N <= 0 || !part || !out) continue;
    if (!job_vec_ok(part, N)) {
      launch_colreduce(part, S, N, out, acc, s, scratch + scr);
      scr += colreduce_scratch_floats(S, N);
      continue;
    }
    CbJob& J = b.j[b.n];
    J.part = part;
    J.out = out;
    J.S = S;
    J.N = N;
    J.accumulate = acc;
    J.strips = S <= CB_SHORT ? (N + CB_SHORT_COLS - 1) / CB_SHORT_COLS : (N + CB_COLS - 1) / CB_COLS;
    J.chunks = S <= CB_SHORT ? 1 : (S + CB_ROWS - 1) / CB_ROWS;
    J.wg0 = wg;
    J.cnt0 = cnt0;
    J.scr0 = scr;
    wg += J.strips * J.chunks;
    if (J.chunks > 1) {
      cnt0 += J.strips;
      scr += (int64_t)J.chunks * N;
    }
    if (++b.n == CB_MAXJ) flush();
  }
  flush();
  VIT_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
