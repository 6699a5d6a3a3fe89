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
