// copy_probe3.hip -- k_push's particle streams with its lane mapping, and
// with a stand-in for its per-block compute between the loads and the stores.
//
// The measured copy ceiling (tools/copy_probe2.hip, "push": 6.09-6.35 TB/s)
// maps a wave instruction to 1 KB of contiguous 16-B vectors.  k_push
// (PINC_PUSH_CONSEC) gives each thread four consecutive particles: its two
// 16-B loads per array sit 16 B apart, so one wave instruction covers every
// other 16 B of 2 KB and the next instruction the rest.  Variants, 6 arrays
// of the C4 species size (3 positions to other arrays, 3 velocities in
// place, one 256-thread block per 1024 particles):
//   contig     copy_probe2's "push" mapping
//   consec     k_push's mapping
//   consec_w   k_push's mapping plus `work` rounds of block-synchronised
//              work between the loads and the stores (an FMA chain per item
//              and an LDS round trip with a barrier per round), standing in
//              for the box, E staging, kick and deposit phases
//   contig_w   the same work on the contiguous mapping
//   consec_pf  consec_w whose blocks, after their loads, touch the next
//              block's lines once (a 4-B load per 128-B line per array,
//              its value folded in) -- a prefetch into L2 ahead of that
//              block's own loads
//
//   hipcc -std=c++17 -O3 --offload-arch=gfx950 tools/copy_probe3.hip -o tools/copy_probe3
//   tools/copy_probe3 [MiB per array = 8192] [reps = 3] [work rounds = 24]
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

struct Arr {
	dvec2 *x[6];
	dvec2 *y[6];
};
constexpr int kBS = 256;
constexpr int kChunk = 512;  // 16-B vectors per array per block (1024 particles)

// MODE 0: contiguous (vector u*256 + t), 1: consecutive pairs (vector 2t + u)
// PF: touch the next block's lines after the loads
template <int MODE, bool WORK, bool PF>
__global__ __launch_bounds__(kBS) void push_streams(Arr a, long n, int work, double *sink) {
	__shared__ double lds[kBS * 2];
	const long b0 = (long)blockIdx.x * kChunk;
	auto vid = [&](int u) -> long { return MODE == 0 ? b0 + u * kBS + threadIdx.x : b0 + 2 * threadIdx.x + u; };
	dvec2 v[6][2];
#pragma unroll
	for (int c = 0; c < 6; c++)
#pragma unroll
		for (int u = 0; u < 2; u++) {
			const long i = vid(u);
			v[c][u] = i < n ? a.x[c][i] : dvec2{0, 0};
		}
	double pf = 0;
	if (PF) {
		// the next block's 6 x 8 KB: 64 lines of 128 B per array, a 4-B load
		// of each (threads 0..63 per array in turn)
		const long nb0 = b0 + kChunk;
		const int line = threadIdx.x & 63, arr = threadIdx.x >> 6;
#pragma unroll
		for (int r = 0; r < 2; r++) {
			const int c = arr + 4 * r;
			if (c < 6) {
				const long i = nb0 + line * 8;
				if (i < n) pf += ((const float *)(a.x[c] + i))[0];
			}
		}
	}
	if (WORK) {
		double acc = pf;
#pragma unroll
		for (int c = 0; c < 6; c++) acc += v[c][0].x * v[c][1].y;
		for (int r = 0; r < work; r++) {
#pragma unroll 4
			for (int q = 0; q < 8; q++) acc = acc * 0.999 + 1e-3;
			lds[threadIdx.x * 2 + (r & 1)] = acc;
			__syncthreads();
			acc += lds[((threadIdx.x + 17 * r) & (kBS - 1)) * 2 + (r & 1)];
		}
		v[0][0].x += acc * 1e-300;
	} else {
		v[0][0].x += pf * 1e-300;
	}
#pragma unroll
	for (int c = 0; c < 6; c++)
#pragma unroll
		for (int u = 0; u < 2; u++) {
			const long i = vid(u);
			dvec2 *o = c >= 3 ? a.x[c] : a.y[c];
			if (i < n) o[i] = v[c][u] + 1.0;
		}
	if (threadIdx.x == 0 && v[1][1].y == -12345.0) sink[0] = v[2][0].x;
}

int main(int argc, char **argv) {
	const long perArray = (argc > 1 ? atol(argv[1]) : 8192L) << 20;
	const int reps = argc > 2 ? atoi(argv[2]) : 3;
	const int work = argc > 3 ? atoi(argv[3]) : 24;
	const long nv = perArray / 16 / kChunk * kChunk;
	Arr a;
	for (int c = 0; c < 6; c++) {
		CHECK(hipMalloc(&a.x[c], nv * 16));
		CHECK(hipMalloc(&a.y[c], nv * 16));
		CHECK(hipMemset(a.x[c], 0, nv * 16));
		CHECK(hipMemset(a.y[c], 0, nv * 16));
	}
	double *sink;
	CHECK(hipMalloc(&sink, 64));
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	const unsigned nb = (unsigned)(nv / kChunk);
	auto timed = [&](const char *name, auto launch) {
		float best = 1e30f, sum = 0;
		for (int r = 0; r < reps; r++) {
			CHECK(hipEventRecord(e0));
			launch();
			CHECK(hipEventRecord(e1));
			CHECK(hipEventSynchronize(e1));
			float ms = 0;
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			if (ms < best) best = ms;
			sum += ms;
		}
		CHECK(hipGetLastError());
		const double moved = 12.0 * nv * 16;
		printf("{\"kernel\": \"%s\", \"work\": %d, \"per_array_MiB\": %ld, \"best_ms\": %.4f, \"mean_ms\": %.4f, "
		       "\"TBs\": %.3f}\n",
		       name, work, perArray >> 20, best, sum / reps, moved / (best * 1e-3) / 1e12);
		fflush(stdout);
	};
	timed("contig", [&] { push_streams<0, false, false><<<nb, kBS>>>(a, nv, work, sink); });
	timed("consec", [&] { push_streams<1, false, false><<<nb, kBS>>>(a, nv, work, sink); });
	timed("contig_w", [&] { push_streams<0, true, false><<<nb, kBS>>>(a, nv, work, sink); });
	timed("consec_w", [&] { push_streams<1, true, false><<<nb, kBS>>>(a, nv, work, sink); });
	timed("consec_pf", [&] { push_streams<1, true, true><<<nb, kBS>>>(a, nv, work, sink); });
	timed("contig", [&] { push_streams<0, false, false><<<nb, kBS>>>(a, nv, work, sink); });
	timed("consec", [&] { push_streams<1, false, false><<<nb, kBS>>>(a, nv, work, sink); });
	CHECK(hipDeviceSynchronize());
	for (int c = 0; c < 6; c++) {
		CHECK(hipFree(a.x[c]));
		CHECK(hipFree(a.y[c]));
	}
	return 0;
}
