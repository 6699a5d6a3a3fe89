// copy_probe2.hip -- why six-stream copies (k_push's SoA particle streams)
// run slower than one-stream copies on MI355X (tools/copy_probe.hip:
// 1 array 5.8-6.0 TB/s, 6 arrays 4.4-5.1 TB/s), at the push's sizes.
//
// Each array is a separate hipMalloc, as pAlloc makes them (pinc_pop.c).
// One block per chunk of the push's size (1024 particles = 512 16-B vectors
// per array), loads of all arrays then stores, nontemporal or not:
//   soa A     A input arrays -> A output arrays (A = 1, 2, 3, 6)
//   push      3 positions -> 3 other arrays, 3 velocities in place (k_push's
//             plain-push streams)
//   aosoa     one input and one output array holding, per chunk of 1024
//             particles, the six components one after the other (48 KiB
//             contiguous per chunk): the same bytes as soa 6 in two streams
//   aosoa_push  the AoSoA form of `push` (positions to the other array,
//             velocities in place)
// Per-array sizes: argv[1] MiB (default 8192: the C4 species' 8.6 GB).
//
//   hipcc -std=c++17 -O3 --offload-arch=gfx950 tools/copy_probe2.hip -o tools/copy_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double dvec2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                  \
	do {                                                                          \
		hipError_t e_ = (x);                                                      \
		if (e_ != hipSuccess) {                                                   \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
			exit(1);                                                              \
		}                                                                         \
	} while (0)

template <bool NT>
__device__ __forceinline__ dvec2 ld(const dvec2 *p) {
	if constexpr (NT) return __builtin_nontemporal_load(p);
	else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(dvec2 *p, dvec2 v) {
	if constexpr (NT) __builtin_nontemporal_store(v, p);
	else *p = v;
}

struct Arr {
	dvec2 *x[6];
	dvec2 *y[6];
};
constexpr int kBS = 256;
constexpr int kChunk = 512;  // vectors per array per block (1024 particles)

// A streams in -> A streams out; INPLACE: arrays 3..5 are written back in place
template <int A, bool NT, bool INPLACE>
__global__ __launch_bounds__(kBS) void soa(Arr a, long n) {
	const long b0 = (long)blockIdx.x * kChunk;
	dvec2 v[A][kChunk / kBS];
#pragma unroll
	for (int c = 0; c < A; c++)
#pragma unroll
		for (int u = 0; u < kChunk / kBS; u++) {
			const long i = b0 + u * kBS + threadIdx.x;
			v[c][u] = i < n ? ld<NT>(a.x[c] + i) : dvec2{0, 0};
		}
#pragma unroll
	for (int c = 0; c < A; c++)
#pragma unroll
		for (int u = 0; u < kChunk / kBS; u++) {
			const long i = b0 + u * kBS + threadIdx.x;
			dvec2 *o = (INPLACE && c >= 3) ? a.x[c] : a.y[c];
			if (i < n) st<NT>(o + i, v[c][u] + 1.0);
		}
}

// AoSoA: chunk b holds components 0..5 of its 1024 particles, 512 vectors each
template <bool NT, bool INPLACE>
__global__ __launch_bounds__(kBS) void aosoa(dvec2 *in, dvec2 *out, long nChunks) {
	const long b0 = (long)blockIdx.x * 6 * kChunk;
	if (blockIdx.x >= nChunks) return;
	dvec2 v[6][kChunk / kBS];
#pragma unroll
	for (int c = 0; c < 6; c++)
#pragma unroll
		for (int u = 0; u < kChunk / kBS; u++) v[c][u] = ld<NT>(in + b0 + c * kChunk + u * kBS + threadIdx.x);
#pragma unroll
	for (int c = 0; c < 6; c++)
#pragma unroll
		for (int u = 0; u < kChunk / kBS; u++) {
			dvec2 *o = (INPLACE && c >= 3) ? in : out;
			st<NT>(o + b0 + c * kChunk + u * kBS + threadIdx.x, v[c][u] + 1.0);
		}
}

int main(int argc, char **argv) {
	const long perArray = (argc > 1 ? atol(argv[1]) : 8192L) << 20;
	const int reps = argc > 2 ? atoi(argv[2]) : 3;
	const long nv = perArray / 16 / kChunk * kChunk;  // vectors per array, whole chunks
	Arr a;
	for (int c = 0; c < 6; c++) {
		CHECK(hipMalloc(&a.x[c], nv * 16));
		CHECK(hipMalloc(&a.y[c], nv * 16));
		CHECK(hipMemset(a.x[c], 0, nv * 16));
		CHECK(hipMemset(a.y[c], 0, nv * 16));
	}
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	auto timed = [&](const char *name, int nt, double moved, auto launch) {
		float best = 1e30f;
		for (int r = 0; r < reps; r++) {
			CHECK(hipEventRecord(e0));
			launch();
			CHECK(hipEventRecord(e1));
			CHECK(hipEventSynchronize(e1));
			float ms = 0;
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			if (ms < best) best = ms;
		}
		CHECK(hipGetLastError());
		printf("{\"kernel\": \"%s\", \"nt\": %d, \"per_array_MiB\": %ld, \"bytes\": %.0f, \"best_ms\": %.4f, "
		       "\"TBs\": %.3f}\n",
		       name, nt, perArray >> 20, moved, best, moved / (best * 1e-3) / 1e12);
		fflush(stdout);
	};
	const unsigned nb = (unsigned)(nv / kChunk);
	for (int nt = 0; nt < 2; nt++) {
#define SOA(A, IP)                                                                                         \
	timed(IP ? "push" : "soa" #A, nt, 2.0 * (A) * nv * 16, [&] {                                            \
		if (nt) soa<A, true, IP><<<nb, kBS>>>(a, nv);                                                       \
		else soa<A, false, IP><<<nb, kBS>>>(a, nv);                                                         \
	})
		SOA(1, false);
		SOA(2, false);
		SOA(3, false);
		SOA(6, false);
		SOA(6, true);
		// AoSoA over the first array pair seen as one buffer of nChunks * 6 * kChunk vectors
		// (x[0] and y[0] hold nv vectors: nv / 6 / kChunk whole AoSoA chunks of the same bytes)
		const long nChunks = nv / (6 * kChunk);
		timed("aosoa", nt, 2.0 * nChunks * 6 * kChunk * 16, [&] {
			if (nt) aosoa<true, false><<<(unsigned)nChunks, kBS>>>(a.x[0], a.y[0], nChunks);
			else aosoa<false, false><<<(unsigned)nChunks, kBS>>>(a.x[0], a.y[0], nChunks);
		});
		timed("aosoa_push", nt, 2.0 * nChunks * 6 * kChunk * 16, [&] {
			if (nt) aosoa<true, true><<<(unsigned)nChunks, kBS>>>(a.x[0], a.y[0], nChunks);
			else aosoa<false, true><<<(unsigned)nChunks, kBS>>>(a.x[0], a.y[0], nChunks);
		});
	}
	CHECK(hipDeviceSynchronize());
	for (int c = 0; c < 6; c++) {
		CHECK(hipFree(a.x[c]));
		CHECK(hipFree(a.y[c]));
	}
	return 0;
}
