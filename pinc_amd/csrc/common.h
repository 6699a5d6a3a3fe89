// common.h -- shared device helpers for the PINC MI355X kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pinc_hip.h"

#define PINC_WAVE 64

namespace pinc {

// error bookkeeping shared by all translation units (runtime.hip)
int set_error(hipError_t e, const char *where);
int check_launch(const char *where);

// storage index of a padded coordinate p (0..T+1) in a periodic dimension
// stored without ghosts (grid.c halo semantics: ghost 0 == T, T+1 == 1)
__device__ __forceinline__ int wrap_pad(int p, int T) {
	int s = p - 1;
	s = (s < 0) ? s + T : s;
	s = (s >= T) ? s - T : s;
	return s;
}

// periodic neighbour in a ghost-free dimension
__device__ __forceinline__ int wrap(int i, int T) {
	return (i < 0) ? i + T : ((i >= T) ? i - T : i);
}

// Grid-stride walk of the point stencils (residual, norm, restriction,
// prolongation, E = -grad phi).  PINC_MG_XCD: the 8 XCDs (block b on XCD b % 8) take
// contiguous eighths of [0, n) and each XCD's blocks sweep theirs in order,
// so the rows and planes a point's stencil reads around it are read by the
// same XCD close in time (one L2), instead of by the XCDs of the blocks of
// the neighbouring rows.  Placement only: the same points, the same
// arithmetic.  Otherwise the plain grid stride.
#ifndef PINC_MG_XCD_WALK
#define PINC_MG_XCD_WALK 1
#endif
struct Walk {
	long g0, g1, step;
};
__device__ __forceinline__ Walk point_walk(long n) {
	const long nt = blockDim.x;
#if PINC_MG_XCD_WALK
	if ((gridDim.x & 7u) == 0) {
		const unsigned x = blockIdx.x & 7u, j = blockIdx.x >> 3, perXcd = gridDim.x >> 3;
		const long span = ((n + 8 * nt - 1) / (8 * nt)) * nt;  // an eighth, whole blocks
		const long b0 = (long)x * span;
		return {b0 + (long)j * nt + threadIdx.x, min(n, b0 + span), (long)perXcd * nt};
	}
#endif
	return {(long)blockIdx.x * nt + threadIdx.x, n, (long)gridDim.x * nt};
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
	return v;
}

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
	const int lane = threadIdx.x & 63;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		T u = __shfl_up(v, o, 64);
		if (lane >= o) v += u;
	}
	return v;
}

// deterministic block sum (fixed shape: blockDim multiple of 64, <=1024)
__device__ __forceinline__ double block_sum(double v, double *lds) {
	v = wave_sum(v);
	int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	if (lane == 0) lds[w] = v;
	__syncthreads();
	double r = 0.;
	if (threadIdx.x == 0) {
		int nw = blockDim.x >> 6;
		for (int i = 0; i < nw; i++) r += lds[i];
	}
	__syncthreads();
	return r;  // valid in thread 0
}

}  // namespace pinc
