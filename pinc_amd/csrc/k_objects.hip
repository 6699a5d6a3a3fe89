// k_objects.hip -- immersed objects (object.c, config C5) on the device.
//
//   pinc_hip_obj_flag      oCollectObjectCharge's test (object.c:481-505): a
//                          particle whose cell's lower node is an interior
//                          node of an object is flagged for removal, in the
//                          emigrant classification format (flag != center),
//                          with per-chunk counts, so the removal itself is
//                          pinc_hip_extract's back-fill (the order the
//                          serial loop gives, the object checker under oracle/)
//   pinc_hip_obj_gather    phi at the surface nodes (object.c:327-333)
//   pinc_hip_obj_correct   eq. 5 (object.c:349-362): rhoCorr_i =
//                          sum_j M[j][i] (phi_c - phi_j), added to rho at the
//                          surface nodes; one thread per surface node i, the
//                          row-major M read along i (coalesced)
//   pinc_hip_obj_add       a constant added at the surface nodes (the
//                          collected charge spread over the surface)
#include <hip/hip_runtime.h>
#include "pinc_hip.h"
#include "common.h"

namespace {

constexpr int kObjThreads = 256;

__global__ __launch_bounds__(kObjThreads) void k_obj_flag(const double *__restrict__ x0,
                                                          const double *__restrict__ x1,
                                                          const double *__restrict__ x2, long n,
                                                          const unsigned char *__restrict__ inside, long sy,
                                                          long sz, long nNodes, int center,
                                                          unsigned char *__restrict__ flags,
                                                          int *__restrict__ chunkCount,
                                                          int *__restrict__ objCount) {
	__shared__ int wcnt[kObjThreads / 64];
	const long base = (long)blockIdx.x * PINC_CHUNK;
	int cnt = 0;
	for (int k = 0; k < PINC_CHUNK / kObjThreads; k++) {
		const long i = base + k * kObjThreads + threadIdx.x;
		if (i >= n) break;
		// object.c:489-494: p = j + k*sizeProd[2] + l*sizeProd[3]
		const long node = (long)(int)x0[i] + (long)(int)x1[i] * sy + (long)(int)x2[i] * sz;
		const int id = (node >= 0 && node < nNodes) ? inside[node] : 0;
		flags[i] = (unsigned char)(id ? 0 : center);
		cnt += id != 0;
		if (id) atomicAdd(&objCount[id - 1], 1);  // rare: particles entering an object
	}
	int wsum = cnt;
	for (int o = 32; o > 0; o >>= 1) wsum += __shfl_xor(wsum, o);
	if ((threadIdx.x & 63) == 0) wcnt[threadIdx.x >> 6] = wsum;
	__syncthreads();
	if (threadIdx.x == 0) {
		int t = 0;
		for (int w = 0; w < kObjThreads / 64; w++) t += wcnt[w];
		chunkCount[blockIdx.x] = t;
	}
}

__global__ void k_obj_gather(const double *__restrict__ grid, const long *__restrict__ idx, long n,
                             double *__restrict__ out) {
	const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) out[i] = idx[i] >= 0 ? grid[idx[i]] : 0.0;  // -1: another rank's node
}

__global__ void k_obj_correct(const double *__restrict__ M, const double *__restrict__ phiS, long n, double phiC,
                              const long *__restrict__ idx, double *__restrict__ rho) {
	const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	double c = 0.0;
	if (idx[i] < 0) return;  // surface node of another rank's slab
	for (long j = 0; j < n; j++) c += M[n * j + i] * (phiC - phiS[j]);
	rho[idx[i]] += c;
}

__global__ void k_obj_add(double *__restrict__ grid, const long *__restrict__ idx, long n, double v) {
	const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n && idx[i] >= 0) grid[idx[i]] += v;
}

int check(const char *what) { return pinc::check_launch(what); }

}  // namespace

extern "C" int pinc_hip_obj_flag(pinc_pop_t pop, int s, const unsigned char *inside, long sy, long sz, long nNodes,
                                 unsigned char *flags, int *chunkCount, int *objCount, void *stream) {
	const long n = pop.iStop[s] - pop.iStart[s];
	if (n <= 0) return 0;
	if (pop.nd != 3) return pinc::set_error(hipErrorInvalidValue, "objects are 3-D (object.c)");
	const long b0 = pop.iStart[s];
	int center = 13;
	hipLaunchKernelGGL(k_obj_flag, dim3((unsigned)((n + PINC_CHUNK - 1) / PINC_CHUNK)), dim3(kObjThreads), 0,
	                   (hipStream_t)stream, pop.x[0] + b0, pop.x[1] + b0, pop.x[2] + b0, n, inside, sy, sz, nNodes,
	                   center, flags + b0, chunkCount, objCount);
	return check("obj flag");
}

extern "C" int pinc_hip_obj_gather(const double *grid, const long *idx, long n, double *out, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_obj_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, grid, idx,
	                   n, out);
	return check("obj gather");
}

extern "C" int pinc_hip_obj_correct(const double *M, const double *phiS, long n, double phiC, const long *idx,
                                    double *rho, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_obj_correct, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, M, phiS,
	                   n, phiC, idx, rho);
	return check("obj correct");
}

extern "C" int pinc_hip_obj_add(double *grid, const long *idx, long n, double v, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_obj_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, grid, idx, n,
	                   v);
	return check("obj add");
}
