// copy_probe.hip -- what HBM copy rate this MI355X reaches, and in which
// load/store form (MI355X_MICROARCH.md quotes 6.29 TB/s
// for a float4 copy; tools/pmc_calibrate.hip's cp_pair32, the push's
// streaming shape, reached 4.77 TB/s).
//
// Every variant copies (reads and writes) a known number of bytes between
// two 2 GiB buffers (8x the Infinity Cache); rate = (read + write bytes) /
// best time of `reps` launches.  Variants:
//   U    16-B vectors per lane per iteration (loads of an iteration issued
//        before its stores: U*16 B in flight per lane)
//   NT   nontemporal loads and stores (global_load/store ... nt)
//   arrays  1 = one array in, one out; 6 = six in, six out (k_push's six
//        SoA streams: x,y,z,vx,vy,vz)
//   grid    grid-stride with G blocks, or "chunk": one block per contiguous
//        chunk of the push's size (blocks = n / chunk, no grid stride)
//
//   hipcc -std=c++17 -O3 --offload-arch=gfx950 tools/copy_probe.hip -o tools/copy_probe
//   ./tools/copy_probe [MiB] [reps]
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
	const dvec2 *x[6];
	dvec2 *y[6];
};

// grid-stride: iteration covers U * blockDim vectors of every array
template <int A, int U, bool NT, int BS>
__global__ __launch_bounds__(BS) void cp_grid(Arr a, long n) {
	const long step = (long)gridDim.x * BS * U;
	for (long base = (long)blockIdx.x * BS * U + threadIdx.x; base < n; base += step) {
		dvec2 v[A][U];
#pragma unroll
		for (int c = 0; c < A; c++)
#pragma unroll
			for (int u = 0; u < U; u++) {
				const long i = base + (long)u * BS;
				v[c][u] = i < n ? ld<NT>(a.x[c] + i) : dvec2{0, 0};
			}
#pragma unroll
		for (int c = 0; c < A; c++)
#pragma unroll
			for (int u = 0; u < U; u++) {
				const long i = base + (long)u * BS;
				if (i < n) st<NT>(a.y[c] + i, v[c][u] + 1.0);
			}
	}
}

// one block per contiguous chunk of `chunk` vectors per array
template <int A, int U, bool NT, int BS>
__global__ __launch_bounds__(BS) void cp_chunk(Arr a, long n, int chunk) {
	const long b0 = (long)blockIdx.x * chunk;
	for (int off = 0; off < chunk; off += BS * U) {
		dvec2 v[A][U];
#pragma unroll
		for (int c = 0; c < A; c++)
#pragma unroll
			for (int u = 0; u < U; u++) {
				const long i = b0 + off + (long)u * BS + threadIdx.x;
				v[c][u] = i < n ? ld<NT>(a.x[c] + i) : dvec2{0, 0};
			}
#pragma unroll
		for (int c = 0; c < A; c++)
#pragma unroll
			for (int u = 0; u < U; u++) {
				const long i = b0 + off + (long)u * BS + threadIdx.x;
				if (i < n) st<NT>(a.y[c] + i, v[c][u] + 1.0);
			}
	}
}

int main(int argc, char **argv) {
	const long bytes = argc > 1 ? atol(argv[1]) << 20 : 2048L << 20;
	const int reps = argc > 2 ? atoi(argv[2]) : 5;
	char *pa, *pb;
	CHECK(hipMalloc(&pa, bytes));
	CHECK(hipMalloc(&pb, bytes));
	CHECK(hipMemset(pa, 0, bytes));
	CHECK(hipMemset(pb, 0, bytes));
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	auto arrays = [&](int A) {
		Arr a;
		const long nv = bytes / 16 / A;
		for (int c = 0; c < 6; c++) {
			a.x[c] = reinterpret_cast<const dvec2 *>(pa) + (c < A ? c : 0) * nv;
			a.y[c] = reinterpret_cast<dvec2 *>(pb) + (c < A ? c : 0) * nv;
		}
		return a;
	};
	auto timed = [&](const char *name, int A, int U, int nt, const char *grid, int bs, long nv, auto launch) {
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
		const double moved = 2.0 * A * nv * 16;
		printf("{\"kernel\": \"%s\", \"arrays\": %d, \"U\": %d, \"nt\": %d, \"grid\": \"%s\", \"block\": %d, "
		       "\"bytes\": %.0f, \"best_ms\": %.4f, \"TBs\": %.3f}\n",
		       name, A, U, nt, grid, bs, moved, best, moved / (best * 1e-3) / 1e12);
		fflush(stdout);
	};
#define GRID(A, U, NT, BS, G)                                                                           \
	do {                                                                                                 \
		Arr a = arrays(A);                                                                               \
		const long nv = bytes / 16 / (A);                                                                \
		char g[32];                                                                                      \
		snprintf(g, sizeof g, "%d", (G));                                                                \
		timed("cp_grid", A, U, NT, g, BS, nv, [&] { cp_grid<A, U, NT, BS><<<(G), BS>>>(a, nv); });       \
	} while (0)
#define CHUNK(A, U, NT, BS, CH)                                                                         \
	do {                                                                                                 \
		Arr a = arrays(A);                                                                               \
		const long nv = bytes / 16 / (A);                                                                \
		char g[32];                                                                                      \
		snprintf(g, sizeof g, "chunk%d", (CH));                                                          \
		timed("cp_chunk", A, U, NT, g, BS, nv,                                                           \
		      [&] { cp_chunk<A, U, NT, BS><<<(unsigned)((nv + (CH) - 1) / (CH)), BS>>>(a, nv, (CH)); }); \
	} while (0)
	// one array: width of work per lane, nontemporal, grid size
	for (int G : {1024, 2048, 4096, 8192}) {
		GRID(1, 1, 0, 256, G);
		GRID(1, 1, 1, 256, G);
		GRID(1, 4, 0, 256, G);
		GRID(1, 4, 1, 256, G);
	}
	GRID(1, 2, 1, 256, 2048);
	GRID(1, 8, 1, 256, 2048);
	GRID(1, 4, 1, 512, 2048);
	GRID(1, 4, 1, 1024, 1024);
	// six arrays (the push's streams)
	for (int G : {1024, 2048, 4096}) {
		GRID(6, 1, 0, 256, G);
		GRID(6, 1, 1, 256, G);
		GRID(6, 2, 1, 256, G);
	}
	// one block per chunk (the push's launch: 1024 particles = 512 vectors per array)
	CHUNK(6, 1, 0, 256, 512);
	CHUNK(6, 1, 1, 256, 512);
	CHUNK(6, 2, 1, 256, 512);
	CHUNK(6, 2, 1, 256, 1024);
	CHUNK(6, 2, 1, 256, 2048);
	CHUNK(1, 4, 1, 256, 4096);
	CHUNK(1, 4, 0, 256, 4096);
	CHECK(hipDeviceSynchronize());
	CHECK(hipFree(pa));
	CHECK(hipFree(pb));
	return 0;
}
