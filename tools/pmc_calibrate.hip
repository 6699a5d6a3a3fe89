// pmc_calibrate.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE
// on gfx950 for the access widths and patterns this repository's kernels
// use (MI355X_MICROARCH.md, HBM: "FETCH_SIZE reports exactly 1/2 of the
// bytes of a wide coalesced streaming read (16 B/lane) ... other access
// widths are uncalibrated: calibrate on a known byte count").
//
// Every kernel touches a known number of bytes of a 2 GiB buffer (8x the
// 256 MiB Infinity Cache, so the bytes reach HBM), once:
//   rd_b32 / rd_b64 / rd_b128  consecutive 4 / 8 / 16 B per lane
//   rd_pair32                  k_push's particle loads: lane l reads 16 B at
//                              32 l and, in a second instruction, 16 B at
//                              32 l + 16 (PINC_PUSH_CONSEC)
//   rd_b64_rows                k_mg's stencil loads: 8 B per lane, each
//                              thread reads its row and the rows +-1 (a
//                              3-row sliding window: every byte is fetched
//                              once from HBM, re-reads hit L2)
//   wr_b64 / wr_b128 / wr_pair32 / wr_b8x4 / at_f64  the matching stores
//                              (wr_b8x4: k_push's flag bytes, lane l writes
//                              4 l .. 4 l + 3 one byte at a time), and
//                              no-return fp64 atomic adds, 8 B per lane
//   cp_pair32                  k_push's streaming shape: read 48 B and write
//                              48 B per particle in the pair32 pattern over
//                              six arrays (the achievable HBM rate of the
//                              push's own bytes, no compute)
// Run it under rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, and
// --kernel-trace --stats (tools/pmc_calibrate.sh); tools/pmc_summary.py
// --calibrate turns the counters into per-pattern correction factors.
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

constexpr int kT = 256;

__global__ __launch_bounds__(kT) void rd_b32(const float *__restrict__ a, long n, float *__restrict__ out) {
	float s = 0;
	for (long i = blockIdx.x * (long)kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) s += a[i];
	if (s == 12345.f) out[0] = s;  // never true for the zero-filled input: keeps the loads
}
__global__ __launch_bounds__(kT) void rd_b64(const double *__restrict__ a, long n, double *__restrict__ out) {
	double s = 0;
	for (long i = blockIdx.x * (long)kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) s += a[i];
	if (s == 12345.0) out[0] = s;
}
__global__ __launch_bounds__(kT) void rd_b128(const dvec2 *__restrict__ a, long n, double *__restrict__ out) {
	double s = 0;
	for (long i = blockIdx.x * (long)kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) {
		dvec2 v = a[i];
		s += v.x + v.y;
	}
	if (s == 12345.0) out[0] = s;
}
// n doubles; each thread reads 4 consecutive doubles as two 16-B loads
__global__ __launch_bounds__(kT) void rd_pair32(const double *__restrict__ a, long n, double *__restrict__ out) {
	double s = 0;
	for (long i = 4 * (blockIdx.x * (long)kT + threadIdx.x); i + 3 < n; i += 4 * (long)gridDim.x * kT) {
		dvec2 v0 = *reinterpret_cast<const dvec2 *>(a + i);
		dvec2 v1 = *reinterpret_cast<const dvec2 *>(a + i + 2);
		s += v0.x + v0.y + v1.x + v1.y;
	}
	if (s == 12345.0) out[0] = s;
}
// rows of W doubles; thread x of a block sweeps rows r0..r1 reading rows
// r-1, r, r+1 at column x (the stencil's z-neighbour reads)
__global__ __launch_bounds__(kT) void rd_b64_rows(const double *__restrict__ a, long rows, int W, int rowsPerBlock,
                                                   double *__restrict__ out) {
	const int cols = W / kT;
	double s = 0;
	for (int c = 0; c < cols; c++) {
		const long x = (long)c * kT + threadIdx.x;
		const long r0 = (long)blockIdx.x * rowsPerBlock;
		for (long r = r0; r < r0 + rowsPerBlock && r < rows; r++) {
			const long rm = r > 0 ? r - 1 : rows - 1, rp = r + 1 < rows ? r + 1 : 0;
			s += a[rm * W + x] + a[r * W + x] + a[rp * W + x];
		}
	}
	if (s == 12345.0) out[0] = s;
}
__global__ __launch_bounds__(kT) void wr_b64(double *__restrict__ a, long n) {
	for (long i = blockIdx.x * (long)kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) a[i] = (double)i;
}
__global__ __launch_bounds__(kT) void wr_b128(dvec2 *__restrict__ a, long n) {
	for (long i = blockIdx.x * (long)kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) a[i] = dvec2{(double)i, 1.0};
}
__global__ __launch_bounds__(kT) void wr_pair32(double *__restrict__ a, long n) {
	for (long i = 4 * (blockIdx.x * (long)kT + threadIdx.x); i + 3 < n; i += 4 * (long)gridDim.x * kT) {
		*reinterpret_cast<dvec2 *>(a + i) = dvec2{(double)i, 1.0};
		*reinterpret_cast<dvec2 *>(a + i + 2) = dvec2{2.0, 3.0};
	}
}
__global__ __launch_bounds__(kT) void wr_b8x4(unsigned char *__restrict__ a, long n) {
	for (long i = 4 * (blockIdx.x * (long)kT + threadIdx.x); i + 3 < n; i += 4 * (long)gridDim.x * kT)
		for (int k = 0; k < 4; k++) a[i + k] = (unsigned char)(i + k);
}
__global__ __launch_bounds__(kT) void at_f64(double *__restrict__ a, long n) {
	for (long i = blockIdx.x * (long)kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) unsafeAtomicAdd(&a[i], 1.0);
}
struct Six {
	const double *x[6];
	double *y[6];
};
__global__ __launch_bounds__(kT) void cp_pair32(Six s, long n) {
	for (long i = 4 * (blockIdx.x * (long)kT + threadIdx.x); i + 3 < n; i += 4 * (long)gridDim.x * kT) {
		dvec2 v[6][2];
#pragma unroll
		for (int c = 0; c < 6; c++) {
			v[c][0] = *reinterpret_cast<const dvec2 *>(s.x[c] + i);
			v[c][1] = *reinterpret_cast<const dvec2 *>(s.x[c] + i + 2);
		}
#pragma unroll
		for (int c = 0; c < 6; c++) {
			*reinterpret_cast<dvec2 *>(s.y[c] + i) = v[c][0] + 1.0;
			*reinterpret_cast<dvec2 *>(s.y[c] + i + 2) = v[c][1] + 1.0;
		}
	}
}

// the push's streaming shape in other patterns: one particle per lane with
// 8-B accesses, two consecutive particles per lane with 16-B accesses, and
// pair32 with the velocities updated in place (the plain push writes its
// positions to the other buffer and its velocities in place)
__global__ __launch_bounds__(kT) void cp_b64(Six s, long n) {
	for (long i = blockIdx.x * (long)kT + threadIdx.x; i < n; i += (long)gridDim.x * kT) {
		double v[6];
#pragma unroll
		for (int c = 0; c < 6; c++) v[c] = s.x[c][i];
#pragma unroll
		for (int c = 0; c < 6; c++) s.y[c][i] = v[c] + 1.0;
	}
}
__global__ __launch_bounds__(kT) void cp_b128(Six s, long n) {
	for (long i = 2 * (blockIdx.x * (long)kT + threadIdx.x); i + 1 < n; i += 2 * (long)gridDim.x * kT) {
		dvec2 v[6];
#pragma unroll
		for (int c = 0; c < 6; c++) v[c] = *reinterpret_cast<const dvec2 *>(s.x[c] + i);
#pragma unroll
		for (int c = 0; c < 6; c++) *reinterpret_cast<dvec2 *>(s.y[c] + i) = v[c] + 1.0;
	}
}
__global__ __launch_bounds__(kT) void cp_push(Six s, long n) {
	// s.y[0..2] positions out, velocities in place in s.x[3..5]
	for (long i = 4 * (blockIdx.x * (long)kT + threadIdx.x); i + 3 < n; i += 4 * (long)gridDim.x * kT) {
		dvec2 v[6][2];
#pragma unroll
		for (int c = 0; c < 6; c++) {
			v[c][0] = *reinterpret_cast<const dvec2 *>(s.x[c] + i);
			v[c][1] = *reinterpret_cast<const dvec2 *>(s.x[c] + i + 2);
		}
#pragma unroll
		for (int c = 0; c < 6; c++) {
			double *o = c < 3 ? s.y[c] : const_cast<double *>(s.x[c]);
			*reinterpret_cast<dvec2 *>(o + i) = v[c][0] + 1.0;
			*reinterpret_cast<dvec2 *>(o + i + 2) = v[c][1] + 1.0;
		}
	}
}

int main(int argc, char **argv) {
	const long bytes = argc > 1 ? atol(argv[1]) << 20 : 2048L << 20;  // MiB
	const int reps = argc > 2 ? atoi(argv[2]) : 3;
	char *a, *b;
	double *out;
	CHECK(hipMalloc(&a, bytes));
	CHECK(hipMalloc(&b, bytes));
	CHECK(hipMalloc(&out, 64));
	CHECK(hipMemset(a, 0, bytes));
	CHECK(hipMemset(b, 0, bytes));
	// cp_pair32: six inputs and six outputs of bytes/6 each inside a and b
	const long n6 = (bytes / 6 / 8) & ~3L;
	Six six;
	for (int c = 0; c < 6; c++) {
		six.x[c] = reinterpret_cast<const double *>(a) + c * n6;
		six.y[c] = reinterpret_cast<double *>(b) + c * n6;
	}
	const int grid = 256 * 16;
	const int W = 1024, rowsPerBlock = 64;
	const long rows = bytes / 8 / W;
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	auto timed = [&](const char *name, double nbytes, auto launch) {
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
		printf("{\"kernel\": \"%s\", \"bytes\": %.0f, \"best_ms\": %.4f, \"GBs\": %.1f}\n", name, nbytes, best,
		       nbytes / (best * 1e-3) / 1e9);
	};
	timed("rd_b32", bytes, [&] { rd_b32<<<grid, kT>>>((const float *)a, bytes / 4, (float *)out); });
	timed("rd_b64", bytes, [&] { rd_b64<<<grid, kT>>>((const double *)a, bytes / 8, out); });
	timed("rd_b128", bytes, [&] { rd_b128<<<grid, kT>>>((const dvec2 *)a, bytes / 16, out); });
	timed("rd_pair32", bytes, [&] { rd_pair32<<<grid, kT>>>((const double *)a, bytes / 8, out); });
	timed("rd_b64_rows", (double)rows * W * 8,
	      [&] { rd_b64_rows<<<(rows + rowsPerBlock - 1) / rowsPerBlock, kT>>>((const double *)a, rows, W, rowsPerBlock, out); });
	timed("wr_b64", bytes, [&] { wr_b64<<<grid, kT>>>((double *)b, bytes / 8); });
	timed("wr_b128", bytes, [&] { wr_b128<<<grid, kT>>>((dvec2 *)b, bytes / 16); });
	timed("wr_pair32", bytes, [&] { wr_pair32<<<grid, kT>>>((double *)b, bytes / 8); });
	timed("wr_b8x4", bytes / 8, [&] { wr_b8x4<<<grid, kT>>>((unsigned char *)b, bytes / 8); });
	timed("at_f64", bytes / 4, [&] { at_f64<<<grid, kT>>>((double *)b, bytes / 4 / 8); });
	timed("cp_pair32", 2.0 * 6 * n6 * 8, [&] { cp_pair32<<<grid, kT>>>(six, n6); });
	timed("cp_b64", 2.0 * 6 * n6 * 8, [&] { cp_b64<<<grid, kT>>>(six, n6); });
	timed("cp_b128", 2.0 * 6 * n6 * 8, [&] { cp_b128<<<grid, kT>>>(six, n6); });
	timed("cp_push", 2.0 * 6 * n6 * 8, [&] { cp_push<<<grid, kT>>>(six, n6); });
	// the same with a grid of one block per 1024 particles (the push's launch)
	timed("cp_pair32_chunks", 2.0 * 6 * n6 * 8, [&] { cp_pair32<<<(unsigned)(n6 / 1024), kT>>>(six, n6); });
	timed("cp_push_chunks", 2.0 * 6 * n6 * 8, [&] { cp_push<<<(unsigned)(n6 / 1024), kT>>>(six, n6); });
	CHECK(hipDeviceSynchronize());
	CHECK(hipFree(a));
	CHECK(hipFree(b));
	CHECK(hipFree(out));
	return 0;
}
