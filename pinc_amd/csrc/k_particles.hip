// k_particles.hip -- particle kernels of the PINC hot path for MI355X (gfx950).
//
//   move + classify     puMove (pusher.c:86-119) fused with the neighbour test
//                       of puExtractEmigrants3D/ND (pusher.c:782-910)
//   extract             the reference's serial back-fill compaction, made
//                       parallel without changing its result or the order in
//                       which emigrants are listed (DESIGN.md "Migration")
//   import              shiftImmigrants + importParticles (pusher.c:941-985)
//   deposit             puDistr3D1 / puDistrND1 (pusher.c:512-638)
//   accelerate          puAcc3D1KE / puAccND1KE + interpolators
//                       (pusher.c:178-265, 1089-1162)
//   init                pPosLattice / pPosPerturb / pVel* (population.c)
//
// All arithmetic is fp64 in the reference's association order; the library
// is compiled with -ffp-contract=off so no multiply-add is fused.
#include "common.h"
#include <type_traits>

using namespace pinc;

namespace {

struct Thr {
	double lo[3], up[3], hi[3];
	int T[3];  // true cells per dimension (local)
};

constexpr int kThreads = 256;
constexpr int kItems = PINC_CHUNK / kThreads;

__device__ __forceinline__ unsigned long long lanemask_lt() {
	return (1ull << (threadIdx.x & 63)) - 1ull;
}

// ------------------------------------------------------------ move --------
template <int ND>
__global__ __launch_bounds__(kThreads) void k_move_classify(
		double *__restrict__ x0, double *__restrict__ x1, double *__restrict__ x2,
		const double *__restrict__ v0, const double *__restrict__ v1,
		const double *__restrict__ v2, long n, int doMove, Thr thr, int center,
		unsigned char *__restrict__ flags, int *__restrict__ chunkCount, double maxVel,
		int *__restrict__ err, int wrapMask) {
	__shared__ int wcnt[kThreads / 64];
	double *xs[3] = {x0, x1, x2};
	const double *vs[3] = {v0, v1, v2};
	long base = (long)blockIdx.x * PINC_CHUNK;
	int cnt = 0;
	int bad = 0;
#pragma unroll 2
	for (int k = 0; k < kItems; k++) {
		long i = base + k * kThreads + threadIdx.x;
		if (i >= n) break;
		double p[ND];
#pragma unroll
		for (int d = 0; d < ND; d++) {
			p[d] = xs[d][i];
			if (doMove) {
				double v = vs[d][i];
				bad |= (v > maxVel);  // pVelAssertMax (population.c:342-365)
				p[d] += v;
				xs[d][i] = p[d];
			}
		}
		int ne = 0;
#pragma unroll
		for (int d = ND - 1; d >= 0; d--) {
			int dig = 1 - (p[d] < thr.lo[d]) + (p[d] >= thr.up[d]);
			// pPosAssertInLocalFrame after the periodic shift (population.c:316-340)
			double q = p[d] - (double)(dig - 1) * (thr.hi[d] - 1.0);
			bad |= (q < 0.0 || q > thr.hi[d]) << 1;
			if ((wrapMask >> d) & 1) {
				// tiled layout: a crossing of a rank-local periodic boundary is
				// applied in place with the import's shift (pusher.c:941-964)
				if (dig != 1) {
					p[d] = p[d] + (double)((1 - dig) * thr.T[d]);
					xs[d][i] = p[d];
				}
				dig = 1;
			}
			ne = ne * 3 + dig;
		}
		flags[i] = (unsigned char)ne;
		cnt += (ne != center);
	}
	if (bad) atomicOr(err, bad);
	int wsum = wave_sum(cnt);
	if ((threadIdx.x & 63) == 0) wcnt[threadIdx.x >> 6] = wsum;
	__syncthreads();
	if (threadIdx.x == 0) {
		int t = 0;
		for (int w = 0; w < kThreads / 64; w++) t += wcnt[w];
		chunkCount[blockIdx.x] = t;
	}
}

// --------------------------------------------------- single-block scans ---
// exclusive scan of in[0..n) into out[0..n], out[n] = total
__global__ __launch_bounds__(1024) void k_scan_single(const int *__restrict__ in,
                                                      int *__restrict__ out, int n) {
	__shared__ long part[1024];
	int t = threadIdx.x;
	int seg = (n + 1023) / 1024;
	int a = t * seg, b = min(n, a + seg);
	long s = 0;
	for (int i = a; i < b; i++) s += in[i];
	part[t] = s;
	__syncthreads();
	for (int o = 1; o < 1024; o <<= 1) {
		long v = (t >= o) ? part[t - o] : 0;
		__syncthreads();
		part[t] += v;
		__syncthreads();
	}
	long run = part[t] - s;
	for (int i = a; i < b; i++) {
		int v = in[i];
		out[i] = (int)run;
		run += v;
	}
	if (t == 1023) out[n] = (int)part[1023];
}

// ----------------------------------------------------------- extract ------
// Per particle j (relative to the species start) with E(j) = emigrants
// before j, n particles, E emigrants, m = n-E survivors:
//   emigrant j<m   is hole number k=E(j)+1
//   survivor j>=m  is tail survivor number r = n-j-E+E(j) (counted from the end)
//   emigrant j>m   is extracted at position n-j
// (derivation: DESIGN.md "Migration"; checked against the serial loop).
__global__ __launch_bounds__(kThreads) void k_extract_a(
		const unsigned char *__restrict__ flags, long n, int center,
		const int *__restrict__ chunkOffset, int nChunks, int *__restrict__ tail,
		int *__restrict__ holes, int *__restrict__ order, int *__restrict__ scratch) {
	__shared__ int wtot[kThreads / 64];
	long E = chunkOffset[nChunks];
	long m = n - E;
	long base = (long)blockIdx.x * PINC_CHUNK;
	int running = chunkOffset[blockIdx.x];
	// a chunk with no emigrants wholly before m has no holes and no tail
	// survivors: nothing to record (most chunks when few particles leave)
	if (chunkOffset[blockIdx.x + 1] == running && base + PINC_CHUNK <= m) return;
	int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	for (int k = 0; k < kItems; k++) {
		long i = base + k * kThreads + threadIdx.x;
		bool in = i < n;
		bool emig = in && flags[i] != center;
		unsigned long long b = __ballot(emig);
		int rw = __popcll(b & lanemask_lt());
		if (lane == 0) wtot[w] = __popcll(b);
		__syncthreads();
		int before = 0, tot = 0;
		for (int q = 0; q < kThreads / 64; q++) {
			before += (q < w) ? wtot[q] : 0;
			tot += wtot[q];
		}
		long Ej = running + before + rw;
		if (in) {
			if (emig) {
				if (i < m) holes[Ej + 1] = (int)i;
				else if (i > m) order[n - i] = (int)i;
			} else if (i >= m) {
				tail[n - i - E + Ej] = (int)i;
			}
			if (i == m) scratch[0] = (int)Ej;  // number of holes
		}
		running += tot;
		__syncthreads();
	}
}

__global__ void k_extract_b(const unsigned char *__restrict__ flags, long n, long E, int center,
                            const int *__restrict__ tail, const int *__restrict__ holes,
                            int *__restrict__ order, const int *__restrict__ scratch) {
	long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
	long m = n - E;
	int h = scratch[0];
	if (q >= 1 && q <= h) {
		long prevT = (q == 1) ? n : tail[q - 1];
		order[n - prevT] = holes[q];
	}
	if (q == 0 && m < n && flags[m] != center) {
		long t = h ? tail[h] : n;
		order[n - t] = (int)m;
	}
}

// per-block direction histogram over the extraction order
constexpr int kRankItems = 4;
constexpr int kRankChunk = kThreads * kRankItems;
constexpr int kMaxNe = PINC_NE_CODES;  // 27 directions + the object sink

__global__ __launch_bounds__(kThreads) void k_rank_hist(const unsigned char *__restrict__ flags,
                                                        const int *__restrict__ order, long E,
                                                        int *__restrict__ blockHist) {
	__shared__ int hist[kMaxNe];
	if (threadIdx.x < kMaxNe) hist[threadIdx.x] = 0;
	__syncthreads();
	long base = (long)blockIdx.x * kRankChunk;
	for (int k = 0; k < kRankItems; k++) {
		long p = base + k * kThreads + threadIdx.x;
		if (p < E) atomicAdd(&hist[flags[order[p]]], 1);
	}
	__syncthreads();
	if (threadIdx.x < kMaxNe) blockHist[(long)blockIdx.x * kMaxNe + threadIdx.x] = hist[threadIdx.x];
}

// exclusive scan per direction over blocks; bases per direction; counts
__global__ __launch_bounds__(kMaxNe * 32) void k_hist_scan(int *__restrict__ blockHist, int nb,
                                                           int *__restrict__ scratch) {
	// scratch[32..32+kMaxNe): base of each direction, scratch[64..64+kMaxNe): count
	__shared__ int tot[kMaxNe];
	int ne = threadIdx.x >> 5, l = threadIdx.x & 31;
	if (ne < kMaxNe && l == 0) {
		int run = 0;
		for (int b = 0; b < nb; b++) {
			int v = blockHist[(long)b * kMaxNe + ne];
			blockHist[(long)b * kMaxNe + ne] = run;
			run += v;
		}
		tot[ne] = run;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		int run = 0;
		for (int q = 0; q < kMaxNe; q++) {
			scratch[32 + q] = run;
			scratch[64 + q] = tot[q];
			run += tot[q];
		}
	}
}

// stable scatter of emigrants into the direction-ordered buffer
__global__ __launch_bounds__(kThreads) void k_rank_scatter(
		unsigned char *__restrict__ flags, const int *__restrict__ order, long E,
		const int *__restrict__ blockHist, const int *__restrict__ scratch, pinc_pop_t pop,
		long sbase, double *__restrict__ buf, long cap, unsigned char *__restrict__ bufNe, int center) {
	__shared__ int waveCnt[kThreads / 64][kMaxNe];
	__shared__ int running[kMaxNe];
	int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	if (threadIdx.x < kMaxNe) running[threadIdx.x] = 0;
	long base = (long)blockIdx.x * kRankChunk;
	for (int k = 0; k < kRankItems; k++) {
		for (int q = threadIdx.x; q < (kThreads / 64) * kMaxNe; q += kThreads)
			(&waveCnt[0][0])[q] = 0;
		__syncthreads();
		long p = base + k * kThreads + threadIdx.x;
		bool in = p < E;
		int j = in ? order[p] : 0;
		int ne = in ? flags[j] : 31;
		// lanes with the same direction (match-any over 5 bits)
		unsigned long long same = __ballot(in);
#pragma unroll
		for (int bit = 0; bit < 5; bit++) {
			unsigned long long bb = __ballot((ne >> bit) & 1);
			same &= ((ne >> bit) & 1) ? bb : ~bb;
		}
		int rw = __popcll(same & lanemask_lt());
		if (in && rw == 0) waveCnt[w][ne] = __popcll(same);
		__syncthreads();
		if (in) {
			int off = running[ne] + rw;
			for (int q = 0; q < w; q++) off += waveCnt[q][ne];
			long dst = (long)scratch[32 + ne] + blockHist[(long)blockIdx.x * kMaxNe + ne] + off;
			long src = sbase + j;
			for (int d = 0; d < pop.nd; d++) {
				buf[d * cap + dst] = pop.x[d][src];
				buf[(3 + d) * cap + dst] = pop.v[d][src];
			}
			bufNe[dst] = (unsigned char)ne;
			flags[j] = (unsigned char)center;  // (read above by this thread only: the species' flags are
			                                   // all the centre again after the extraction)
		}
		__syncthreads();
		if (threadIdx.x < kMaxNe) {
			int t = 0;
			for (int q = 0; q < kThreads / 64; q++) t += waveCnt[q][threadIdx.x];
			running[threadIdx.x] += t;
		}
		__syncthreads();
	}
}

__global__ void k_fill_holes(pinc_pop_t pop, long sbase, const int *__restrict__ tail,
                             const int *__restrict__ holes, const int *__restrict__ scratch) {
	long k = (long)blockIdx.x * blockDim.x + threadIdx.x + 1;
	int h = scratch[0];
	if (k > h) return;
	long src = sbase + tail[k], dst = sbase + holes[k];
	for (int d = 0; d < pop.nd; d++) {
		pop.x[d][dst] = pop.x[d][src];
		pop.v[d][dst] = pop.v[d][src];
	}
}

__global__ void k_import(pinc_pop_t pop, long dst, const double *__restrict__ buf, long cap,
                         const unsigned char *__restrict__ bufNe, long first, long n, int T0,
                         int T1, int T2, int shiftMask) {
	long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
	if (q >= n) return;
	long e = first + q;
	int ne = bufNe[e];
	int T[3] = {T0, T1, T2};
	for (int d = 0; d < pop.nd; d++) {
		int dig = ne % 3;
		ne /= 3;
		// receiver tag t = reciprocal(ne): shift = (digit_d(t)-1)*T_d = (1-dig)*T_d
		double shift = ((shiftMask >> d) & 1) ? (double)((1 - dig) * T[d]) : 0.0;
		pop.x[d][dst + q] = buf[d * cap + e] + shift;
		pop.v[d][dst + q] = buf[(3 + d) * cap + e];
	}
}

__global__ void k_pack(const double *__restrict__ buf, long cap, const unsigned char *__restrict__ bufNe,
                       long first, long n, int nd, double *__restrict__ out) {
	long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
	if (q >= n) return;
	long e = first + q;
	double *r = out + q * PINC_REC;
	for (int d = 0; d < 3; d++) {
		r[d] = d < nd ? buf[d * cap + e] : 0.0;
		r[3 + d] = d < nd ? buf[(3 + d) * cap + e] : 0.0;
	}
	r[6] = (double)bufNe[e];
}

__global__ void k_import_rec(pinc_pop_t pop, long dst, const double *__restrict__ rec, long n, int T0,
                             int T1, int T2) {
	long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
	if (q >= n) return;
	const double *r = rec + q * PINC_REC;
	int ne = (int)r[6];
	int T[3] = {T0, T1, T2};
	for (int d = 0; d < pop.nd; d++) {
		int dig = ne % 3;
		ne /= 3;
		pop.x[d][dst + q] = r[d] + (double)((1 - dig) * T[d]);
		pop.v[d][dst + q] = r[3 + d];
	}
}

// ---------------------------------------------------------- deposit -------
struct Geo {
	int T[3];      // storage extent per dim (slab dim: nloc)
	long stride[3];
	int slab;      // slab dimension
};

__device__ __forceinline__ Geo make_geo(const pinc_geom_t &g) {
	// fully unrolled: no dynamically indexed register arrays (scratch)
	Geo r;
	r.slab = g.nd - 1;
	long s = 1;
#pragma unroll
	for (int d = 0; d < 3; d++) {
		r.T[d] = (d == r.slab) ? g.nloc : g.T[d];
		r.stride[d] = s;
		if (d < g.nd) s *= (d == r.slab) ? (long)(g.nloc + 2) : (long)r.T[d];
	}
	return r;
}

// storage coordinate of padded node coordinate p in dim d
__device__ __forceinline__ long node_off(const Geo &G, int d, int p) {
	int s = (d == G.slab) ? p : wrap_pad(p, G.T[d]);
	return (long)s * G.stride[d];
}

// --------------------------------------------- LDS-privatised deposit -----
// One workgroup owns a chunk of kDepChunk consecutive particles; each thread
// owns kDepItems consecutive ones (loaded 16 B at a time).  In either layout
// (the reference's order, spatially coherent from the lattice start, or the
// cell-sorted tiled layout) consecutive particles mostly share a cell and a
// chunk covers a small box of nodes:
//  * a thread sums the eight weights of a run of particles in one cell in
//    registers and adds them once (cell-sorted: once per kDepItems);
//  * the box is accumulated in LDS (ds_add_f64) and flushed with one global
//    atomic per touched node.
// Chunks whose box exceeds the LDS tile use the same run accumulation with
// global atomics.  Weights are the reference's expressions (pusher.c:550-565,
// 626-638); only the summation order differs from the serial loop.
constexpr int kDepItems = 16;
constexpr int kDepChunk = kThreads * kDepItems;
constexpr int kDepCap = 4096;  // LDS nodes per workgroup (32 KiB)

// Integer wave reductions with DPP (row shifts 1, 2, 4, 8, then the row
// broadcasts of lanes 15 and 31): six VALU instructions with DPP operands and
// one readlane, the total uniform.  (The shfl_xor butterflies they replace
// cost six ds_bpermute round trips through the LDS unit each: in the push,
// where nine reductions per block ran that way, a third of its LDS
// instructions.)  Every lane of the wave must be active.
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_i(int old, int v) {
	return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWS, 0xf, false);
}
template <typename Op>
__device__ __forceinline__ int wave_reduce_i(int v, int id, Op op) {
	v = op(v, dpp_i<0x111, 0xf>(id, v));  // row_shr:1
	v = op(v, dpp_i<0x112, 0xf>(id, v));  // row_shr:2
	v = op(v, dpp_i<0x114, 0xf>(id, v));  // row_shr:4
	v = op(v, dpp_i<0x118, 0xf>(id, v));  // row_shr:8 (lane 15 of a row: its total)
	v = op(v, dpp_i<0x142, 0xa>(id, v));  // row_bcast:15 into rows 1, 3
	v = op(v, dpp_i<0x143, 0xc>(id, v));  // row_bcast:31 into rows 2, 3
	return __builtin_amdgcn_readlane(v, 63);
}
#ifndef PINC_DPP_REDUCE
#define PINC_DPP_REDUCE 1
#endif
// fp64 wave sum, the same DPP pattern on the two halves of each partner
// value (a fixed tree: deterministic); the total in every lane's return
__device__ __forceinline__ double wave_sum_d(double v) {
	auto step = [](double x, auto ctrl) -> double {
		constexpr int C = decltype(ctrl)::value >> 4, R = decltype(ctrl)::value & 15;
		const unsigned long long u = __double_as_longlong(x);
		const unsigned lo = __builtin_amdgcn_update_dpp(0u, (unsigned)u, C, R, 0xf, false);
		const unsigned hi = __builtin_amdgcn_update_dpp(0u, (unsigned)(u >> 32), C, R, 0xf, false);
		return x + __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
	};
	v = step(v, std::integral_constant<int, (0x111 << 4) | 0xf>{});
	v = step(v, std::integral_constant<int, (0x112 << 4) | 0xf>{});
	v = step(v, std::integral_constant<int, (0x114 << 4) | 0xf>{});
	v = step(v, std::integral_constant<int, (0x118 << 4) | 0xf>{});
	v = step(v, std::integral_constant<int, (0x142 << 4) | 0xa>{});
	v = step(v, std::integral_constant<int, (0x143 << 4) | 0xc>{});
	const unsigned long long u = __double_as_longlong(v);
	const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, 63), hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), 63);
	return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
#if PINC_DPP_REDUCE
__device__ __forceinline__ int wave_min_i(int v) {
	return wave_reduce_i(v, INT32_MAX, [](int a, int b) { return min(a, b); });
}
__device__ __forceinline__ int wave_max_i(int v) {
	return wave_reduce_i(v, INT32_MIN, [](int a, int b) { return max(a, b); });
}
__device__ __forceinline__ int wave_sum_i(int v) {
	return wave_reduce_i(v, 0, [](int a, int b) { return a + b; });
}
#else
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
	return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
	return v;
}
__device__ __forceinline__ int wave_sum_i(int v) { return wave_sum(v); }
#endif

template <int ND, bool V3D>
__device__ __forceinline__ void cic_weights(const double *dec, const double *comp, double *w) {
	if (V3D) {
		double xc = comp[0], yc = comp[1], zc = comp[2];
		double x = dec[0], y = dec[1], z = dec[2];
		w[0] = xc * yc * zc;
		w[1] = x * yc * zc;
		w[2] = xc * y * zc;
		w[3] = x * y * zc;
		w[4] = xc * yc * z;
		w[5] = x * yc * z;
		w[6] = xc * y * z;
		w[7] = x * y * z;
	} else {
#pragma unroll
		for (int c = 0; c < (1 << ND); c++) {
			double f = 1.0;
#pragma unroll
			for (int d = ND - 1; d >= 1; d--) f = (((c >> d) & 1) ? dec[d] : comp[d]) * f;
			w[c] = ((c & 1) ? dec[0] : comp[0]) * f;
		}
	}
}

// main.c's literal loop adds rho's ghost layers twice (main.c:226,232): a
// weight that lands on a periodic ghost node counts 2^g times, g = its ghost
// coordinates (checked against grid.c:340-406 applied twice).  Slab ghost
// planes are kept on the device and folded twice by the caller; here the
// non-slab dimensions, which are wrapped at deposit, get their factor.
// literal == 2 is the second fold of a deposit made without that factor
// (main.c's loop calling gHaloOp(addSlice, rho, FROMHALO) twice on a library
// that was not told in advance, pinc_grid.c): the weight still missing,
// (2^g_xy - 1) w, and twice that on a slab ghost plane, which the second fold
// adds once more.
template <int ND>
__device__ __forceinline__ double literal_node_factor(const pinc_geom_t &g, const int *p) {
	const int slab = g.nd - 1;
	double m = 1.0, mz = 1.0;
#pragma unroll
	for (int d = 0; d < ND; d++) {
		if (d == slab) {
			if (g.literal == 2 && (p[d] == 0 || p[d] == g.nloc + 1)) mz = 2.0;
			continue;
		}
		if (p[d] == 0 || p[d] == g.T[d] + 1) m *= 2.0;
	}
	return g.literal == 2 ? (m - 1.0) * mz : m;
}

template <int ND>
__device__ __forceinline__ void literal_ghost_weights(const pinc_geom_t &g, const int *j, double *w) {
	if (!g.literal) return;
#pragma unroll
	for (int c = 0; c < (1 << ND); c++) {
		int p[3];
#pragma unroll
		for (int d = 0; d < ND; d++) p[d] = j[d] + ((c >> d) & 1);
		w[c] *= literal_node_factor<ND>(g, p);
	}
}

// global offset of padded node (j[0]+c0, j[1]+c1, ...) for corner c
template <int ND>
__device__ __forceinline__ long corner_off(const Geo &G, const int *j, int c) {
	long off = 0;
#pragma unroll
	for (int d = 0; d < ND; d++) off += node_off(G, d, j[d] + ((c >> d) & 1));
	return off;
}

template <int ND, bool V3D>
__global__ __launch_bounds__(kThreads) void k_deposit_tiled(const double *__restrict__ x0,
                                                            const double *__restrict__ x1,
                                                            const double *__restrict__ x2, long b0,
                                                            long n, pinc_geom_t g,
                                                            double *__restrict__ rho) {
	constexpr int NC = 1 << ND;
	__shared__ double acc[kDepCap];
	__shared__ int red[2 * 3 * (kThreads / 64)];
	__shared__ int box[7];
	Geo G = make_geo(g);
	const double *xs[3] = {x0, x1, x2};
	const long end = b0 + n;
	// thread's items: i0 .. i0+kDepItems-1, i0 even relative to the 16-B
	// aligned base below b0
	const long i0 = (b0 & ~1L) + (long)blockIdx.x * kDepChunk + (long)threadIdx.x * kDepItems;
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	auto load2 = [&](int d, int k, double &a, double &b) {
		long i = i0 + k;
		if (i >= b0 && i + 1 < end) {
			double2 v = *reinterpret_cast<const double2 *>(xs[d] + i);
			a = v.x;
			b = v.y;
		} else {
			a = (i >= b0 && i < end) ? xs[d][i] : 0.0;
			b = (i + 1 >= b0 && i + 1 < end) ? xs[d][i + 1] : 0.0;
		}
	};
	unsigned valid = 0;
#pragma unroll
	for (int k = 0; k < kDepItems; k++) valid |= (unsigned)(i0 + k >= b0 && i0 + k < end) << k;

	// pass 1: bounding box of the chunk's cells (j .. j+1 per dimension)
	int lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
#pragma unroll
	for (int d = 0; d < ND; d++) {
#pragma unroll
		for (int k = 0; k < kDepItems; k += 2) {
			double a, b;
			load2(d, k, a, b);
			if ((valid >> k) & 1u) {
				lo[d] = min(lo[d], (int)a);
				hi[d] = max(hi[d], (int)a + 1);
			}
			if ((valid >> (k + 1)) & 1u) {
				lo[d] = min(lo[d], (int)b);
				hi[d] = max(hi[d], (int)b + 1);
			}
		}
	}
#pragma unroll
	for (int d = 0; d < ND; d++) {
		int a = wave_min_i(lo[d]), b = wave_max_i(hi[d]);
		if (lane == 0) {
			red[(2 * d) * (kThreads / 64) + wv] = a;
			red[(2 * d + 1) * (kThreads / 64) + wv] = b;
		}
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		long vol = 1;
		for (int d = 0; d < ND; d++) {
			int a = INT32_MAX, b = INT32_MIN;
			for (int w = 0; w < kThreads / 64; w++) {
				a = min(a, red[(2 * d) * (kThreads / 64) + w]);
				b = max(b, red[(2 * d + 1) * (kThreads / 64) + w]);
			}
			box[d] = a;
			box[3 + d] = b - a + 1;
			vol *= (long)(b - a + 1);
		}
		box[6] = (vol <= kDepCap && vol > 0) ? (int)vol : 0;
	}
	__syncthreads();
	const int vol = box[6];

	int blo[3] = {0, 0, 0}, st[3] = {0, 0, 0}, bn[3] = {1, 1, 1};
	if (vol) {
		int sz = 1;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			blo[d] = box[d];
			bn[d] = box[3 + d];
			st[d] = sz;
			sz *= bn[d];
		}
		for (int t = threadIdx.x; t < vol; t += kThreads) acc[t] = 0.0;
		__syncthreads();
	}
	int coff[NC];
#pragma unroll
	for (int c = 0; c < NC; c++) {
		coff[c] = 0;
#pragma unroll
		for (int d = 0; d < ND; d++) coff[c] += ((c >> d) & 1) ? st[d] : 0;
	}

	// pass 2: runs of equal cells summed in registers
	int cj[3] = {INT32_MIN, 0, 0};
	double a[NC];
#pragma unroll
	for (int c = 0; c < NC; c++) a[c] = 0.0;
	auto flush = [&]() {
		if (cj[0] == INT32_MIN) return;
		if (vol) {
			int l0 = 0;
#pragma unroll
			for (int d = 0; d < ND; d++) l0 += (cj[d] - blo[d]) * st[d];
#pragma unroll
			for (int c = 0; c < NC; c++) atomicAdd(&acc[l0 + coff[c]], a[c]);
		} else {
#pragma unroll
			for (int c = 0; c < NC; c++) unsafeAtomicAdd(&rho[corner_off<ND>(G, cj, c)], a[c]);
		}
	};
#pragma unroll 2
	for (int k = 0; k < kDepItems; k += 2) {
		double pp[3][2];
#pragma unroll
		for (int d = 0; d < ND; d++) load2(d, k, pp[d][0], pp[d][1]);
#pragma unroll
		for (int h = 0; h < 2; h++) {
			if (!((valid >> (k + h)) & 1u)) continue;
			double dec[3], comp[3], w[NC];
			int j[3];
			bool same = true;
#pragma unroll
			for (int d = 0; d < ND; d++) {
				j[d] = (int)pp[d][h];
				dec[d] = pp[d][h] - j[d];
				comp[d] = 1 - dec[d];
				same = same && (j[d] == cj[d]);
			}
			cic_weights<ND, V3D>(dec, comp, w);
			literal_ghost_weights<ND>(g, j, w);
			if (same) {
#pragma unroll
				for (int c = 0; c < NC; c++) a[c] += w[c];
			} else {
				flush();
#pragma unroll
				for (int c = 0; c < NC; c++) a[c] = w[c];
#pragma unroll
				for (int d = 0; d < ND; d++) cj[d] = j[d];
			}
		}
	}
	flush();
	if (!vol) return;
	__syncthreads();

	// flush the tile: one global atomic per touched node
	for (int t = threadIdx.x; t < vol; t += kThreads) {
		double v = acc[t];
		if (v == 0.0) continue;
		int r = t;
		long off = 0;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			int c = r % bn[d];
			r /= bn[d];
			off += node_off(G, d, blo[d] + c);
		}
		unsafeAtomicAdd(&rho[off], v);
	}
}

// ------------------------------------------------------- accelerate -------
// puAcc3D1KE / puAccND1KE.  The reference rescales the whole E grid per
// species (gMul(E,q/m) ... gMul(E,m/q), pusher.c:192,212); k_field_chain
// materialises E as it stands while species s is pushed (same rounding
// chain), so the particle kernel gathers plain values.  Particles are loaded
// and stored as lane-contiguous 16-B pairs; the gathered corner values are
// reused while a thread's next particle stays in the same cell.
constexpr int kAccItems = 8;
constexpr int kAccChunk = kThreads * kAccItems;

__global__ void k_field_chain(const double *__restrict__ E, double *__restrict__ Es, long n,
                              const double *__restrict__ qm, const double *__restrict__ mq,
                              double pre, int s) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
		double v = E[i] * pre;
		for (int t = 0; t < s; t++) v = (v * qm[t]) * mq[t];
		Es[i] = v * qm[s];
	}
}

// every species' rescaled copy of E in one pass over E (k_field_chain's
// chain for species s is species s-1's times mq[s-1] qm[s] / qm[s-1]... in
// the same expression order: the running v of the loop above), species s at
// Es + s n
__global__ void k_field_chain_all(const double *__restrict__ E, double *__restrict__ Es, long n,
                                  const double *__restrict__ qm, const double *__restrict__ mq, double pre,
                                  int nSpecies) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
		double v = E[i] * pre;
		Es[i] = v * qm[0];
		for (int s = 1; s < nSpecies; s++) {
			v = (v * qm[s - 1]) * mq[s - 1];
			Es[(long)s * n + i] = v * qm[s];
		}
	}
}

// Boris rotation parameters of one species (puGet3DRotationParameters,
// pusher.c:485-505)
struct BorisRot {
	double T[3], S[3];
};

// v x b added to res in addCross's expression order (pusher.c:1234-1238)
__device__ __forceinline__ void add_cross(const double *a, const double *b, double *res) {
	res[0] += (a[1] * b[2] - a[2] * b[1]);
	res[1] += -(a[0] * b[2] - a[2] * b[0]);
	res[2] += (a[0] * b[1] - a[1] * b[0]);
}

template <int ND, bool V3D, bool KE, bool BORIS = false>
__global__ __launch_bounds__(kThreads) void k_accel(const double *__restrict__ x0,
                                                    const double *__restrict__ x1,
                                                    const double *__restrict__ x2,
                                                    double *__restrict__ v0, double *__restrict__ v1,
                                                    double *__restrict__ v2, long b0, long n,
                                                    pinc_geom_t g, const double *__restrict__ E,
                                                    double *__restrict__ kePartial, BorisRot rot = {}) {
	constexpr int NC = 1 << ND;
	__shared__ double red[kThreads / 64];
	Geo G = make_geo(g);
	const double *xs[3] = {x0, x1, x2};
	double *vs[3] = {v0, v1, v2};
	const long end = b0 + n;
	// pair k/2 of the lane-contiguous pairs (1 KiB per wave load instruction)
	const long cb = (b0 & ~1L) + (long)blockIdx.x * kAccChunk + 2L * threadIdx.x;
	double ke = 0.;
	int cj[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
	double e[NC][ND];  // corner values of the current cell
#pragma unroll
	for (int k = 0; k < kAccItems; k += 2) {
		double p[3][2], v[3][2];
		bool ok[2];
		ok[0] = (cb + 2L * kThreads * (k >> 1) >= b0) && (cb + 2L * kThreads * (k >> 1) < end);
		ok[1] = (cb + 2L * kThreads * (k >> 1) + 1 >= b0) && (cb + 2L * kThreads * (k >> 1) + 1 < end);
		if (!ok[0] && !ok[1]) continue;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			if (ok[0] && ok[1]) {
				double2 a = *reinterpret_cast<const double2 *>(xs[d] + cb + 2L * kThreads * (k >> 1));
				double2 b = *reinterpret_cast<const double2 *>(vs[d] + cb + 2L * kThreads * (k >> 1));
				p[d][0] = a.x;
				p[d][1] = a.y;
				v[d][0] = b.x;
				v[d][1] = b.y;
			} else {
				long i = ok[0] ? cb + 2L * kThreads * (k >> 1) : cb + 2L * kThreads * (k >> 1) + 1;
				int h = ok[0] ? 0 : 1;
				p[d][h] = xs[d][i];
				v[d][h] = vs[d][i];
				p[d][1 - h] = p[d][h];
				v[d][1 - h] = v[d][h];
			}
		}
#pragma unroll
		for (int h = 0; h < 2; h++) {
			if (!ok[h]) continue;
			double dec[3], comp[3];
			int j[3];
			bool same = true;
#pragma unroll
			for (int d = 0; d < ND; d++) {
				j[d] = (int)p[d][h];
				dec[d] = p[d][h] - j[d];
				comp[d] = 1 - dec[d];
				same = same && (j[d] == cj[d]);
			}
			if (!same) {
#pragma unroll
				for (int c = 0; c < NC; c++) {
					long off = 0;
#pragma unroll
					for (int d = 0; d < ND; d++) off += node_off(G, d, j[d] + ((c >> d) & 1));
					off *= ND;
#pragma unroll
					for (int q = 0; q < ND; q++) e[c][q] = E[off + q];
				}
#pragma unroll
				for (int d = 0; d < ND; d++) cj[d] = j[d];
			}
			double dv[ND];
			if (V3D) {
				// puInterp3D1 (pusher.c:1116-1120), corner c = x + 2y + 4z
				double x = dec[0], y = dec[1], z = dec[2];
				double xc = comp[0], yc = comp[1], zc = comp[2];
#pragma unroll
				for (int q = 0; q < ND; q++)
					dv[q] = zc * (yc * (xc * e[0][q] + x * e[1][q]) + y * (xc * e[2][q] + x * e[3][q])) +
					        z * (yc * (xc * e[4][q] + x * e[5][q]) + y * (xc * e[6][q] + x * e[7][q]));
			} else {
				// puInterpND1Inner: corner by corner in the recursion order
				// (outer dims first), (c_x*f)*val
#pragma unroll
				for (int q = 0; q < ND; q++) dv[q] = 0;
#pragma unroll
				for (int c = 0; c < (1 << (ND - 1)); c++) {
					double f = 1.0;
					int cc = 0;
#pragma unroll
					for (int d = ND - 1; d >= 1; d--) {
						int bit = (c >> (d - 1)) & 1;
						f = (bit ? dec[d] : comp[d]) * f;
						cc |= bit << d;
					}
#pragma unroll
					for (int q = 0; q < ND; q++) {
						dv[q] += comp[0] * f * e[cc][q];
						dv[q] += dec[0] * f * e[cc | 1][q];
					}
				}
			}
			double vsq = 0;
			if constexpr (BORIS) {
				// puBoris3D1KE (pusher.c:455-476) with the indexing corrected:
				// half kick, rotation about B, KE of v+, half kick
				double vm[3], vp[3];
#pragma unroll
				for (int d = 0; d < 3; d++) vm[d] = v[d][h] + 0.5 * dv[d];
#pragma unroll
				for (int d = 0; d < 3; d++) vp[d] = vm[d];
				add_cross(vm, rot.T, vp);
				add_cross(vp, rot.S, vm);
#pragma unroll
				for (int d = 0; d < 3; d++) vsq += vm[d] * vm[d];
#pragma unroll
				for (int d = 0; d < 3; d++) v[d][h] = vm[d] + 0.5 * dv[d];
			} else {
#pragma unroll
				for (int d = 0; d < ND; d++) {
					double vv = v[d][h];
					vsq += vv * (vv + dv[d]);
					v[d][h] = vv + dv[d];
				}
			}
			ke += vsq;
		}
#pragma unroll
		for (int d = 0; d < ND; d++) {
			if (ok[0] && ok[1]) {
				*reinterpret_cast<double2 *>(vs[d] + cb + 2L * kThreads * (k >> 1)) = make_double2(v[d][0], v[d][1]);
			} else {
				if (ok[0]) vs[d][cb + 2L * kThreads * (k >> 1)] = v[d][0];
				if (ok[1]) vs[d][cb + 2L * kThreads * (k >> 1) + 1] = v[d][1];
			}
		}
	}
	if (KE) {
		double t = block_sum(ke, red);
		if (threadIdx.x == 0) kePartial[blockIdx.x] = t;
	}
}

// ------------------------------------------------------------- init -------
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
	z += 0x9E3779B97F4A7C15ULL;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}
__device__ __forceinline__ double uni(unsigned long long seed, unsigned long long c) {
	unsigned long long x = mix64(seed ^ mix64(c));
	return ((double)(x >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ double normal(unsigned long long seed, unsigned long long c) {
	double u1 = uni(seed, 2 * c), u2 = uni(seed, 2 * c + 1);
	return sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2);
}

struct LatticeArgs {
	int nd;
	int L[3];
	int sub[3];
	int off[3];
	double posToSub[3];
	double l;
	double amp[3], mode[3];
	int perturb, maxwell;
	double drift, vth;
	unsigned long long seed;
	int species;
};

__device__ __forceinline__ bool lattice_pos(const LatticeArgs &a, long i, double *x) {
	double lin = a.l * (double)i;
	for (int d = 0; d < a.nd; d++) {
		x[d] = fmod(lin, (double)a.L[d]);
		lin /= a.L[d];
	}
	int ok = 0;
	for (int d = 0; d < a.nd; d++) ok += (a.sub[d] == (int)(a.posToSub[d] * x[d]));
	return ok == a.nd;
}

__global__ __launch_bounds__(kThreads) void k_lattice_count(LatticeArgs a, long nGlobal,
                                                            int *__restrict__ chunkCount) {
	__shared__ int wcnt[kThreads / 64];
	long base = (long)blockIdx.x * PINC_CHUNK;
	int cnt = 0;
	for (int k = 0; k < kItems; k++) {
		long i = base + k * kThreads + threadIdx.x;
		double x[3];
		if (i < nGlobal && lattice_pos(a, i, x)) cnt++;
	}
	int ws = wave_sum(cnt);
	if ((threadIdx.x & 63) == 0) wcnt[threadIdx.x >> 6] = ws;
	__syncthreads();
	if (threadIdx.x == 0) {
		int t = 0;
		for (int q = 0; q < kThreads / 64; q++) t += wcnt[q];
		chunkCount[blockIdx.x] = t;
	}
}

__global__ __launch_bounds__(kThreads) void k_lattice_write(LatticeArgs a, long nGlobal,
                                                            const int *__restrict__ chunkOffset,
                                                            pinc_pop_t pop, long sbase) {
	__shared__ int wtot[kThreads / 64];
	long base = (long)blockIdx.x * PINC_CHUNK;
	int running = chunkOffset[blockIdx.x];
	int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	for (int k = 0; k < kItems; k++) {
		long i = base + k * kThreads + threadIdx.x;
		double x[3] = {0, 0, 0};
		bool keep = i < nGlobal && lattice_pos(a, i, x);
		unsigned long long b = __ballot(keep);
		int rw = __popcll(b & lanemask_lt());
		if (lane == 0) wtot[w] = __popcll(b);
		__syncthreads();
		int before = 0, tot = 0;
		for (int q = 0; q < kThreads / 64; q++) {
			before += (q < w) ? wtot[q] : 0;
			tot += wtot[q];
		}
		if (keep) {
			long dst = sbase + running + before + rw;
			for (int d = 0; d < a.nd; d++) {
				double p = x[d];  // global frame
				if (a.perturb) {
					double theta = 2.0 * M_PI * a.mode[d] * p / a.L[d];
					p += a.amp[d] * cos(theta);
				}
				pop.x[d][dst] = p - a.off[d];
				double v = 0.0;
				if (a.maxwell) {
					unsigned long long c =
						(((unsigned long long)a.species << 40) | (unsigned long long)i) * 3ULL + d;
					v = a.drift + a.vth * normal(a.seed, c);
				}
				pop.v[d][dst] = v;
			}
		}
		running += tot;
		__syncthreads();
	}
}

inline long ceil_div(long a, long b) { return (a + b - 1) / b; }


// ----------------------------------------------------- tiled layout -------
// Counting sort of one species by tile (a TW^nd block of cells) for the
// optional tiled layout (population:layout = tiled).  Particles of a tile
// become contiguous, so a deposit or gather chunk touches a few hundred
// nodes instead of whole rows.  Within a tile the order is arbitrary.
struct TileGeo {
	int tw;         // cells per tile side
	int nt[3];      // tiles per dimension (cell index (int)p is in [0, T+1])
	int cmax[3];    // largest admissible cell index
	// bricks of the push's sort: tw^(nd-1) consecutive cell keys of a tile
	// (tw x tw x 1 in 3-D), bs[d] = log2 of the brick's extent along d (all
	// 0: bricks of one cell)
	int bs[3];
};

// Sort key: tile index, then the cell inside the tile.  Tiles run along a
// serpentine (x rows alternate direction, y columns alternate per z plane),
// and a tile's layers along the slab dimension run in reverse in odd tiles,
// so consecutive keys of different tiles are neighbouring cells: a block of
// particles that straddles two tiles after a sort spans two adjacent bricks
// (8 x 4 x 1 cells), not a jump of a whole tile row or of the tile's depth.
// Inside a layer the cells are x fastest, so a brick (one layer of a tile,
// TileGeo::bs) is a run of consecutive keys.
template <int ND>
__device__ __forceinline__ long tile_serp(const TileGeo &tg, const int *t) {
	if (ND == 1) return t[0];
	if (ND == 2) return (long)t[1] * tg.nt[0] + ((t[1] & 1) ? tg.nt[0] - 1 - t[0] : t[0]);
	const int ty = (t[2] & 1) ? tg.nt[1] - 1 - t[1] : t[1];
	const long r = (long)t[2] * tg.nt[1] + ty;
	return r * tg.nt[0] + ((r & 1) ? tg.nt[0] - 1 - t[0] : t[0]);
}
// inverse of tile_serp
template <int ND>
__device__ __forceinline__ void tile_unserp(const TileGeo &tg, long tile, int *t) {
	t[1] = t[2] = 0;
	if (ND == 1) {
		t[0] = (int)tile;
		return;
	}
	const long r = tile / tg.nt[0];
	const int tx = (int)(tile - r * tg.nt[0]);
	t[0] = (r & 1) ? tg.nt[0] - 1 - tx : tx;
	if (ND == 2) {
		t[1] = (int)r;
		return;
	}
	t[2] = (int)(r / tg.nt[1]);
	const int ty = (int)(r - (long)t[2] * tg.nt[1]);
	t[1] = (t[2] & 1) ? tg.nt[1] - 1 - ty : ty;
}
// key of clamped cell coordinates c (each in [0, cmax])
template <int ND>
__device__ __forceinline__ int tile_key_of(const TileGeo &tg, const int *c) {
	int t[3] = {0, 0, 0}, in[3] = {0, 0, 0};
#pragma unroll
	for (int d = 0; d < ND; d++) {
		t[d] = c[d] / tg.tw;
		in[d] = c[d] - t[d] * tg.tw;
	}
	const long tile = tile_serp<ND>(tg, t);
	if (ND > 1 && (tile & 1)) in[ND - 1] = tg.tw - 1 - in[ND - 1];
	int cell = 0, cs = 1;
#pragma unroll
	for (int d = 0; d < ND; d++) {
		cell += in[d] * cs;
		cs *= tg.tw;
	}
	return (int)(tile * cs + cell);
}
// cell coordinates of a key (inverse of tile_key_of)
template <int ND>
__device__ __forceinline__ void tile_key_cell(const TileGeo &tg, long key, int *c) {
	int cpt = 1;
#pragma unroll
	for (int d = 0; d < ND; d++) cpt *= tg.tw;
	const long tile = key / cpt;
	int in = (int)(key - tile * cpt);
	int t[3];
	tile_unserp<ND>(tg, tile, t);
	c[1] = c[2] = 0;
#pragma unroll
	for (int d = 0; d < ND; d++) {
		int q = in % tg.tw;
		in /= tg.tw;
		if (ND > 1 && d == ND - 1 && (tile & 1)) q = tg.tw - 1 - q;
		c[d] = t[d] * tg.tw + q;
	}
}
template <int ND>
__device__ __forceinline__ int tile_key(const TileGeo &tg, const double *p) {
	int c[3] = {0, 0, 0};
#pragma unroll
	for (int d = 0; d < ND; d++) {
		const int x = (int)p[d];
		c[d] = x < 0 ? 0 : (x > tg.cmax[d] ? tg.cmax[d] : x);
	}
	return tile_key_of<ND>(tg, c);
}

// wave-aggregated atomicAdd of 1 per active lane on ctr[key]; returns the
// lane's slot (old value + rank among the lanes with the same key)
__device__ __forceinline__ int agg_add(int *ctr, int key, bool active) {
	int lane = threadIdx.x & 63;
	unsigned long long pending = __ballot(active);
	int mine = 0;
	while (pending) {
		int leader = __ffsll((long long)pending) - 1;
		int lk = __shfl(key, leader, 64);
		unsigned long long m = __ballot(active && key == lk) & pending;
		int base = 0;
		if (lane == leader) base = atomicAdd(&ctr[lk], __popcll(m));
		base = __shfl(base, leader, 64);
		if ((m >> lane) & 1ull) mine = base + __popcll(m & lanemask_lt());
		pending &= ~m;
	}
	return mine;
}

template <int ND>
__global__ __launch_bounds__(kThreads) void k_sort_count(const double *__restrict__ x0,
                                                         const double *__restrict__ x1,
                                                         const double *__restrict__ x2, long n,
                                                         TileGeo tg, int *__restrict__ counts) {
	const double *xs[3] = {x0, x1, x2};
	for (long base = (long)blockIdx.x * blockDim.x; base < n; base += (long)gridDim.x * blockDim.x) {
		long i = base + threadIdx.x;
		bool act = i < n;
		double p[3] = {0, 0, 0};
		if (act) {
#pragma unroll
			for (int d = 0; d < ND; d++) p[d] = xs[d][i];
		}
		int key = act ? tile_key<ND>(tg, p) : 0;
		agg_add(counts, key, act);
	}
}

// the sorting push's key counts: per brick, at the brick's first key (the
// push reserves per brick; immigrants joining the counts, or counts made
// without a counting push)
// Cell a particle is sorted by in the in-push sort (the counting push, the
// brick counts and the sorting push must agree): with PINC_SORT_AHEAD (the
// default) the cell of x + v, where the next push's drift takes it before its
// kick, so that a sorting push's output lies in the bricks it was ranked
// into (sorted by the input cell x, the output of every block spread one
// cell around its bricks: E and charge boxes 6 x 6 x 3 cells instead of
// 4 x 4 x 1).  Clamped to the grid like every key (a particle that wraps
// through a periodic face is placed at the face it left: order only).
#ifndef PINC_SORT_AHEAD
#define PINC_SORT_AHEAD 1
#endif
__device__ __forceinline__ int sort_cell(double x, double v) { return PINC_SORT_AHEAD ? (int)(x + v) : (int)x; }

template <int ND>
__global__ __launch_bounds__(kThreads) void k_count_bricks(const double *__restrict__ x0,
                                                           const double *__restrict__ x1,
                                                           const double *__restrict__ x2,
                                                           const double *__restrict__ v0,
                                                           const double *__restrict__ v1,
                                                           const double *__restrict__ v2, long n,
                                                           TileGeo tg, int *__restrict__ counts) {
	const double *xs[3] = {x0, x1, x2}, *vs[3] = {v0, v1, v2};
	for (long base = (long)blockIdx.x * blockDim.x; base < n; base += (long)gridDim.x * blockDim.x) {
		long i = base + threadIdx.x;
		bool act = i < n;
		int c[3] = {0, 0, 0};
		if (act) {
#pragma unroll
			for (int d = 0; d < ND; d++) c[d] = sort_cell(xs[d][i], vs[d][i]);
		}
		agg_add(counts, act ? brick_first_key<ND>(tg, c) : 0, act);
	}
}

template <int ND>
__global__ __launch_bounds__(kThreads) void k_sort_scatter(pinc_pop_t in, pinc_pop_t out, long b0, long n,
                                                           TileGeo tg, int *__restrict__ cursor) {
	for (long base = (long)blockIdx.x * blockDim.x; base < n; base += (long)gridDim.x * blockDim.x) {
		long i = base + threadIdx.x;
		bool act = i < n;
		double p[3] = {0, 0, 0}, v[3] = {0, 0, 0};
		if (act) {
#pragma unroll
			for (int d = 0; d < ND; d++) {
				p[d] = in.x[d][b0 + i];
				v[d] = in.v[d][b0 + i];
			}
		}
		int key = act ? tile_key<ND>(tg, p) : 0;
		int slot = agg_add(cursor, key, act);
		if (act) {
#pragma unroll
			for (int d = 0; d < ND; d++) {
				out.x[d][b0 + slot] = p[d];
				out.v[d][b0 + slot] = v[d];
			}
		}
	}
}


// exclusive scan of n ints for large n: block sums, a single-block scan of
// those, then per-block scans with the block offsets; out[n] = total
constexpr int kScanItems = 16;
constexpr int kScanBlock = kThreads * kScanItems;

__global__ __launch_bounds__(kThreads) void k_scan_sums(const int *__restrict__ in, long n,
                                                        int *__restrict__ sums) {
	__shared__ int w[kThreads / 64];
	long b0 = (long)blockIdx.x * kScanBlock;
	int t = 0;
	for (int k = 0; k < kScanItems; k++) {
		long i = b0 + (long)k * kThreads + threadIdx.x;
		if (i < n) t += in[i];
	}
	t = wave_sum(t);
	if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = t;
	__syncthreads();
	if (threadIdx.x == 0) {
		int s = 0;
		for (int q = 0; q < kThreads / 64; q++) s += w[q];
		sums[blockIdx.x] = s;
	}
}

__global__ __launch_bounds__(kThreads) void k_scan_apply(const int *__restrict__ in, long n,
                                                         const int *__restrict__ offs,
                                                         int *__restrict__ out) {
	__shared__ int wtot[kThreads / 64];
	long b0 = (long)blockIdx.x * kScanBlock;
	// thread owns kScanItems consecutive elements
	long i0 = b0 + (long)threadIdx.x * kScanItems;
	int v[kScanItems];
	int t = 0;
#pragma unroll
	for (int k = 0; k < kScanItems; k++) {
		v[k] = (i0 + k < n) ? in[i0 + k] : 0;
		t += v[k];
	}
	// exclusive scan of t over the block
	int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	int x = t;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		int y = __shfl_up(x, o, 64);
		if (lane >= o) x += y;
	}
	if (lane == 63) wtot[wv] = x;
	__syncthreads();
	int before = 0;
	for (int q = 0; q < wv; q++) before += wtot[q];
	int run = offs[blockIdx.x] + before + x - t;
#pragma unroll
	for (int k = 0; k < kScanItems; k++) {
		if (i0 + k < n) out[i0 + k] = run;
		run += v[k];
	}
	if (i0 + kScanItems >= n && i0 < n) out[n] = run;
}


// ------------------------------------------ deposit over sorted cell ranges --
// Tiled layout after a sort: offs is the sort's cursor array after the
// scatter, i.e. the exclusive end of each key's range, so [offs[key-1],
// offs[key]) holds the particles that were in cell `key` at the last sort.  One thread per cell
// sums the eight CIC weights of its particles in registers (no atomics per
// particle); particles that have since moved to another cell are added
// individually (LDS box with a one-cell margin, else global atomics).  A
// workgroup covers 256 consecutive keys (4 tiles in 3-D), accumulated in LDS
// and flushed once.
template <int ND, bool V3D>
__global__ __launch_bounds__(kThreads) void k_deposit_cells(const double *__restrict__ x0,
                                                            const double *__restrict__ x1,
                                                            const double *__restrict__ x2, long nCell,
                                                            const int *__restrict__ offs, long nKeys,
                                                            TileGeo tg, pinc_geom_t g,
                                                            double *__restrict__ rho) {
	constexpr int NC = 1 << ND;
	__shared__ double acc[kDepCap];
	Geo G = make_geo(g);
	const double *xs[3] = {x0, x1, x2};
	int cpt = 1;
#pragma unroll
	for (int d = 0; d < ND; d++) cpt *= tg.tw;
	const long k0 = (long)blockIdx.x * kThreads;
	const long k1 = min(k0 + kThreads, nKeys) - 1;
	// node box of the block's tiles plus a one-cell margin (the tiles of a
	// key range are a path of neighbouring tiles, tile_serp)
	const long t0 = k0 / cpt, t1 = k1 / cpt;
	int tlo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, thi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
	for (long t = t0; t <= t1; t++) {
		int tc[3];
		tile_unserp<ND>(tg, t, tc);
#pragma unroll
		for (int d = 0; d < ND; d++) {
			tlo[d] = min(tlo[d], tc[d]);
			thi[d] = max(thi[d], tc[d]);
		}
	}
	const bool boxOk = t1 - t0 < 16;
	int blo[3] = {0, 0, 0}, bn[3] = {1, 1, 1}, st[3] = {0, 0, 0};
	int vol = 1;
#pragma unroll
	for (int d = 0; d < ND; d++) {
		int clo = tlo[d] * tg.tw, chi = min(thi[d] * tg.tw + tg.tw - 1, tg.cmax[d]);
		blo[d] = clo - 1;
		bn[d] = chi - clo + 4;  // nodes clo-1 .. chi+2
		st[d] = vol;
		vol *= bn[d];
	}
	if (!boxOk || vol > kDepCap) vol = 0;
	for (int t = threadIdx.x; t < vol; t += kThreads) acc[t] = 0.0;
	__syncthreads();

	auto add8 = [&](const int *j, const double *w) {
		bool inBox = vol > 0;
#pragma unroll
		for (int d = 0; d < ND; d++) inBox = inBox && j[d] >= blo[d] && j[d] + 1 < blo[d] + bn[d];
		if (inBox) {
			int l0 = 0;
#pragma unroll
			for (int d = 0; d < ND; d++) l0 += (j[d] - blo[d]) * st[d];
#pragma unroll
			for (int c = 0; c < NC; c++) {
				int off = l0;
#pragma unroll
				for (int d = 0; d < ND; d++) off += ((c >> d) & 1) ? st[d] : 0;
				atomicAdd(&acc[off], w[c]);
			}
		} else {
#pragma unroll
			for (int c = 0; c < NC; c++) unsafeAtomicAdd(&rho[corner_off<ND>(G, j, c)], w[c]);
		}
	};

	const long key = k0 + threadIdx.x;
	if (key < nKeys) {
		// this thread's cell
		int cell[3] = {0, 0, 0};
		tile_key_cell<ND>(tg, key, cell);
		long a = key > 0 ? (long)offs[key - 1] : 0, b = min((long)offs[key], nCell);
		double sum[NC];
#pragma unroll
		for (int c = 0; c < NC; c++) sum[c] = 0.0;
		bool any = false;
		for (long i = a; i < b; i++) {
			double dec[3], comp[3], w[NC];
			int j[3];
			bool own = true;
#pragma unroll
			for (int d = 0; d < ND; d++) {
				double p = xs[d][i];
				j[d] = (int)p;
				dec[d] = p - j[d];
				comp[d] = 1 - dec[d];
				own = own && j[d] == cell[d];
			}
			cic_weights<ND, V3D>(dec, comp, w);
			literal_ghost_weights<ND>(g, j, w);
			if (own) {
#pragma unroll
				for (int c = 0; c < NC; c++) sum[c] += w[c];
				any = true;
			} else {
				add8(j, w);
			}
		}
		if (any) add8(cell, sum);
	}
	if (!vol) return;
	__syncthreads();
	for (int t = threadIdx.x; t < vol; t += kThreads) {
		double v = acc[t];
		if (v == 0.0) continue;
		int r = t;
		long off = 0;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			int c = r % bn[d];
			r /= bn[d];
			off += node_off(G, d, blo[d] + c);
		}
		unsafeAtomicAdd(&rho[off], v);
	}
}

// ------------------------------------------------------- fused push -------
// One pass over a species: [kick: puAcc gather + v += dv + KE (pusher.c:
// 178-265, 1089-1162)] then drift: puMove (pusher.c:86-119) + the neighbour
// test of puExtractEmigrants (pusher.c:782-910) + puDistr of every particle
// that stays (pusher.c:512-638).  Particles that emigrate are deposited after
// their import (distr's immigrant pass), so the charge is the reference's.
//
// Thread t of block b owns particles b*2048 + k*256 + t (k = 0..7): every
// wave load and store is one contiguous 512-B run.  In a cell-ordered layout
// the 64 particles of a wave share one or two cells, so the deposit first
// reduces each large same-cell group across the wave (a transposed butterfly
// that leaves corner c's sum in lane 8c) and adds it once; the other lanes
// (particles that changed cell, sparse groups) add their own eight weights.
// Adds go to an LDS box of the block's cells (ds_add_f64), flushed with one
// global atomic per touched node; a block whose box exceeds the LDS tile adds
// to global memory directly.  Only the summation order differs from the
// serial loop.
struct PushArgs {
	const double *xi[3];
	double *xo[3];       // may alias xi (unsorted)
	const double *vi[3];
	double *vo[3];       // may alias vi (unsorted)
	long n;              // particles of the species; pointers start at it
	pinc_geom_t g;
	const double *Es;    // kick: E as rescaled for the species (k_field_chain)
	double *rho;         // species charge accumulator (slab layout)
	Thr thr;
	int center, wrapMask;
	double maxVel;
	unsigned char *flags;
	int *chunkCount;
	int *err;
	double *kePartial;
	// sorted output (tiled layout): particle i goes to cursor[key(x_i)]++,
	// the keys of the moved particles are counted in cntNext for the next push
	TileGeo tg;
	int *cursor;
	int *cntNext;
	unsigned long long *moved;  // += particles that stay but changed cell (nullable)
	unsigned long long *spread;  // += the block's input cell-box volume (nullable)
	unsigned long long *tstamp;  // 8 phase timestamps per block (diagnostics, nullable)
	unsigned long long *diag;    // [0] += sorting-push items given a global slot one by one (nullable)
	const unsigned char *objIn;  // object ids of the padded nodes (nullable: no objects)
	long objSy, objSz, objN;
	int *objCount;
	int objLo[3], objExt[3];     // bounding box of the object nodes: lower corner, extent - 1
	unsigned long long *emigTotal;  // += particles flagged to leave (nullable)
	int flagsSparse;                // only the non-centre flags are written
};
// phase timestamp of the block (thread 0, s_memrealtime at 100 MHz)
#define PUSH_TS(slot) \
	if (a.tstamp && threadIdx.x == 0) a.tstamp[(long)chunk * 8 + (slot)] = tsub = wall_clock64()
// sub-phase of the sorting push since the last PUSH_TS / PUSH_SUB, summed over
// the blocks into diag[k] (trace mode)
#define PUSH_SUB(k)                                                           \
	if (a.tstamp && threadIdx.x == 0) {                                       \
		const unsigned long long now = wall_clock64();                        \
		atomicAdd(&a.diag[k], now - tsub);                                    \
		tsub = now;                                                           \
	}

// same-cell groups of at least kPushGroupMin lanes (at most kPushGroups of
// them per wave and item) are summed across the wave before the LDS add
// (6: measured at C4, 30.34 ms per species launch against 30.84 with 2;
// smaller groups are cheaper as direct LDS adds than as wave reductions)
#ifndef PINC_PUSH_GROUP_MIN
#define PINC_PUSH_GROUP_MIN 6
#endif
#ifndef PINC_PUSH_GROUPS
#define PINC_PUSH_GROUPS 4
#endif
constexpr int kPushGroupMin = PINC_PUSH_GROUP_MIN;
// diagnostics only (timing by elimination, wrong results): bit 0 skips the
// deposit, bit 1 the E staging and gather, bit 2 the flush
#ifndef PINC_PUSH_SKIP
#define PINC_PUSH_SKIP 0
#endif
// deposit into per-lane-group copies of the LDS charge box (lane & (nc-1)
// picks the copy, nc <= PINC_PUSH_COPIES copies as the box allows) with
// plain LDS atomics, instead of same-cell wave reductions (0).  Measured at
// C4 (mean over the sort cycle): 0 copies 29.6 ms per species launch,
// 2 copies 30.0, 4 copies 28.2, 8 copies 28.2 -- a sorted wave's lanes
// mostly share one cell, and 8 copies cut the same-address conflicts of
// each ds_add_f64 to 8-way for ~60 fewer VALU instructions per particle
// than the reduction.  (Tried and rejected the same day: whole-chunk
// launches without per-element conditions, 43 ms, spills; 2 items per
// thread at 4-5 waves/SIMD, 31-32 ms; 512-thread blocks, 35.8 ms.)
#ifndef PINC_PUSH_COPIES
#define PINC_PUSH_COPIES 8
#endif
// 1: a thread's particles are consecutive in memory, with plain loads and
// stores (measured at C4, mean over the sort cycle, per species launch:
// 27.1 ms against 28.3 for lane pairs 512 apart with nontemporal access;
// this pattern with nontemporal loads and stores 42 ms, nontemporal stores
// only 33.7, nontemporal loads only 30.1 -- each wave instruction covers
// every other 16 B of 2 KB and the next one the rest, which must meet in
// L2; PMC traffic 122 GB per launch against 110 GB)
#ifndef PINC_PUSH_CONSEC
#define PINC_PUSH_CONSEC 1
#endif
// lane pairs (PINC_PUSH_CONSEC 0): nontemporal particle loads and stores
#ifndef PINC_PUSH_NT
#define PINC_PUSH_NT 0
#endif
// 1 (with PINC_PUSH_CONSEC): a full block's particle loads and stores are
// contiguous per wave instruction (lane l: 16-B pair l, then pair 64 + l of
// the wave's 256 particles) and adjacent lanes swap one pair each (DPP), so
// that a thread still holds four consecutive particles: even lane 2k those
// at 4k, odd lane 2k + 1 those at 128 + 4k.  The mapping where a thread
// loads its own four (every other 16 B of 2 KB per instruction) copies at
// 5.69 TB/s on this chip against 6.13 TB/s contiguous
// (profiles/r06b_copy_probe3_lane_mapping.jsonl)
#ifndef PINC_PUSH_XCH
#define PINC_PUSH_XCH 2
#endif
// (PINC_PUSH_XCH 2, full blocks) bit 0: nontemporal particle loads, bit 1:
// nontemporal particle stores (every wave instruction covers whole lines).
// Both (3): plain push 19.63 -> 19.06 ms per species launch at C4, loads
// alone 19.39, stores alone 19.30 (profiles/r06g_push_nontemporal_ab.txt);
// with the round-5 mapping, where two instructions shared each line,
// nontemporal access was slower (27.1 -> 30.1-42 ms, round 2)
#ifndef PINC_PUSH_XCH_NT
#define PINC_PUSH_XCH_NT 3
#endif
// 1: the counting push adds a thread's same-brick items with one plain LDS
// atomic instead of wave-aggregated adds per item (counting push 22.36 ->
// 21.79 ms at C4, plain push unchanged, no spill with the lane exchange's
// registers; profiles/r06i_count_runs_sort_nt_ab.txt)
#ifndef PINC_PUSH_COUNT_RUNS
#define PINC_PUSH_COUNT_RUNS 1
#endif
#ifndef PINC_PUSH_RHO_LDS
#define PINC_PUSH_RHO_LDS 2048
#endif
constexpr int kRhoLds = PINC_PUSH_COPIES ? PINC_PUSH_RHO_LDS : 1024;

constexpr int kPushGroups = PINC_PUSH_GROUPS;
// 8 waves x 4 particles per thread per PINC_CHUNK block: fewer live VGPRs
// (px) than 4 waves x 8, so more waves per SIMD hide the gather latency
#ifndef PINC_PUSH_ITEMS
#define PINC_PUSH_ITEMS 4
#endif
#ifndef PINC_PUSH_WPE
#define PINC_PUSH_WPE 4
#endif
// 2 (default): pieces of PINC_PUSH_XCD_PIECE chunks round-robin over the
// XCDs (C4: step 55.39 -> 55.07 ms; the contiguous eighths of 1 left the XCD
// holding the top z tiles 1.2 ms behind the others on the electrons)
#ifndef PINC_PUSH_XCD
#define PINC_PUSH_XCD 2
#endif
#ifndef PINC_PUSH_XCD_PIECE
#define PINC_PUSH_XCD_PIECE 64
#endif
#ifndef PINC_PUSH_THREADS
#define PINC_PUSH_THREADS 256
#endif
// 1: the sorting push orders each brick's run by cell (per (brick, cell)
// counters for blocks whose brick box holds at most kCellRankBricks bricks of
// at most 16 cells), so repeated sorts keep a brick's particles cell-contiguous
#ifndef PINC_SORT_CELLRANK
#define PINC_SORT_CELLRANK 1
#endif
constexpr int kCellRankBricks = 64;
// wave priority (s_setprio) of a block's particle-load phase (> 0), or of
// everything after it (< 0); 0: off
#ifndef PINC_PUSH_PRIO
#define PINC_PUSH_PRIO 0
#endif
// 1: per-item periodic images only in blocks that straddle a boundary (k_push)
#ifndef PINC_PUSH_IMG_GATE
#define PINC_PUSH_IMG_GATE 1
#endif
// 1: the cell-change statistic from the pre-move cell, the frame test only
// for particles that leave the centre (k_push)
#ifndef PINC_PUSH_LEAN
#define PINC_PUSH_LEAN 1
#endif
constexpr int kPushThreads = PINC_PUSH_THREADS;
constexpr int kPushItems = PINC_PUSH_ITEMS;  // particles per thread, in lane-contiguous pairs
constexpr int kPushChunk = kPushThreads * kPushItems;  // particles per block (PINC_CHUNK / 2 by default)
static_assert(kPushChunk >= PINC_CHUNK / 8 && PINC_CHUNK % kPushChunk == 0, "kePartial holds PINC_CHUNK/8 per chunk");

// double-precision lane exchange helpers on the two 32-bit halves
__device__ __forceinline__ void permlane32_swap(double &a, double &b) {
	// v_permlane32_swap_b32: lanes 32..63 of a <-> lanes 0..31 of b
	unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
	auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
	auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
	a = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
	b = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}
__device__ __forceinline__ void permlane16_swap(double &a, double &b) {
	// v_permlane16_swap_b32: odd rows of a <-> even rows of b (rows of 16 lanes)
	unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
	auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
	auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
	a = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
	b = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
	unsigned long long u = __double_as_longlong(v);
	unsigned lo = __builtin_amdgcn_update_dpp(0u, (unsigned)u, CTRL, 0xf, 0xf, false);
	unsigned hi = __builtin_amdgcn_update_dpp(0u, (unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
	return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
constexpr int kDppRowRor8 = 0x128, kDppHalfMirror = 0x141, kDppQuadXor2 = 0x4e, kDppQuadXor1 = 0xb1;

// sum of r[0..7] over the 64 lanes, transposed: afterwards lane l holds the
// total of corner 4*b5 + 2*b4 + b3 (b = bits of l) in lanes with (l & 7) == 0
__device__ __forceinline__ double wave_reduce8(double *r) {
	const int lane = threadIdx.x & 63;
	// lanes 0..31 gather corners 0..3, lanes 32..63 corners 4..7
	double a[4];
#pragma unroll
	for (int i = 0; i < 4; i++) {
		double x = r[i], y = r[i + 4];
		permlane32_swap(x, y);
		a[i] = x + y;
	}
	// rows 0,2 gather a[0..1], rows 1,3 a[2..3]
	double b[2];
#pragma unroll
	for (int i = 0; i < 2; i++) {
		double x = a[i], y = a[i + 2];
		permlane16_swap(x, y);
		b[i] = x + y;
	}
	// half rows: lanes with bit 3 clear keep b[0], set keep b[1]
	const bool h3 = lane & 8;
	double send = h3 ? b[0] : b[1];
	double keep = h3 ? b[1] : b[0];
	double c = keep + dpp<kDppRowRor8>(send);
	// total over the 8 lanes of each group
	c += dpp<kDppHalfMirror>(c);
	c += dpp<kDppQuadXor2>(c);
	c += dpp<kDppQuadXor1>(c);
	return c;
}

// storage offsets (in nodes, 32-bit) of padded node coordinates j and j+1
// along dimension d of the slab (periodic x/y stored without ghosts)
struct Geo32 {
	int T[3];
	int stride[3];
	int slab;
};
__device__ __forceinline__ Geo32 make_geo32(const pinc_geom_t &g) {
	Geo32 r;
	r.slab = g.nd - 1;
	int s = 1;
#pragma unroll
	for (int d = 0; d < 3; d++) {
		r.T[d] = (d == r.slab) ? g.nloc : g.T[d];
		r.stride[d] = s;
		if (d < g.nd) s *= (d == r.slab) ? (g.nloc + 2) : r.T[d];
	}
	return r;
}
// (node coordinates and strides are < 2^24: 24-bit multiplies, full rate)
__device__ __forceinline__ int mul24(int a, int b) { return (int)__umul24((unsigned)a, (unsigned)b); }
__device__ __forceinline__ void node_pair(const Geo32 &G, int d, int j, int &o0, int &o1) {
	if (d == G.slab) {
		o0 = d ? mul24(j, G.stride[d]) : j;
		o1 = o0 + G.stride[d];
	} else {
		// wrap_pad of j and j+1 (padded coordinates 0..T+1; a periodic image
		// of the block's boxes may lie one period either side, -T < j < 2T)
		int s0 = j - 1, s1 = j;
		s0 = s0 < 0 ? s0 + G.T[d] : (s0 >= G.T[d] ? s0 - G.T[d] : s0);
		s1 = s1 < 0 ? s1 + G.T[d] : (s1 >= G.T[d] ? s1 - G.T[d] : s1);
		o0 = d ? mul24(s0, G.stride[d]) : s0;
		o1 = d ? mul24(s1, G.stride[d]) : s1;
	}
}
// periodic images of the cells nearest to the block's reference cell r (the
// cell of its first item).  The half cells 0 and T (thresholds at 0.5 and
// T + 0.5) are one cell of the torus: a particle that crosses T + 0.5 lands
// in cell 0 while its neighbours stay in cell T, and the block's boxes,
// centred on the mean cell, would sit between the two.  E at image nodes is
// the same data (wrapped storage; the slab's ghost planes when the slab
// dimension wraps, whose images stay within cells 0..T).  Block-uniform
// bounds: cells <= lo move up by T, cells >= hi down by T.
struct Images {
	int lo[3], hi[3], T[3];
	__device__ __forceinline__ int operator()(int d, int c) const {
		return c + (c <= lo[d] ? T[d] : 0) - (c >= hi[d] ? T[d] : 0);
	}
};
__device__ __forceinline__ Images make_images(const Geo32 &G, int wrapMask, const int *r, int nd) {
	Images m;
	for (int d = 0; d < 3; d++) {
		const int T = G.T[d], h = T / 2;
		m.T[d] = T;
		m.lo[d] = INT32_MIN;
		m.hi[d] = INT32_MAX;
		if (d >= nd) continue;
		if (d != G.slab) {
			m.lo[d] = r[d] - h - 1;
			m.hi[d] = r[d] + h + 1;
		} else if ((wrapMask >> d) & 1) {
			m.lo[d] = min(r[d] - h - 1, 0);
			m.hi[d] = max(r[d] + h + 1, T);
		}
	}
	return m;
}

// LDS capacities of the push: E nodes (pre-move cells + 1), charge nodes
// (post-move cells + 1), input cells and output cells of the sort counters
// (the sorting push, whose LDS also holds the rank array, keeps the smaller
// charge box).  The unsorted push's boxes take a chunk that straddles
// two tiles (8 x 4 x 4 cells) after a step of motion ((10 x 6 x 6 cells):
// 539 E nodes, 1053 charge nodes); with 384 and 1024 such chunks -- a
// quarter of them -- gathered E and added charge through global memory.
constexpr int kRhoBoxCap = 1024;
#ifndef PINC_PUSH_EBOX
#define PINC_PUSH_EBOX 768
#endif
constexpr int kEBoxCapPlain = PINC_PUSH_EBOX;
#ifndef PINC_PUSH_SORT_EBOX
#define PINC_PUSH_SORT_EBOX PINC_PUSH_EBOX
#endif
constexpr int kEBoxCapSort = PINC_PUSH_SORT_EBOX;
constexpr int kInCellCap = 256;
constexpr int kOutCellCap = 512;

// box of integer coordinates: origin, extents, volume, linear index
struct Box {
	int lo[3], n[3];
	int vol;
	__device__ __forceinline__ int index(const int *c, int nd) const {
		int l = 0, s = 1;
		for (int d = 0; d < nd; d++) {
			l += mul24(c[d] - lo[d], s);
			s *= n[d];
		}
		return l;
	}
	__device__ __forceinline__ bool inside(const int *c, int nd) const {
		bool ok = vol > 0;
		for (int d = 0; d < nd; d++) ok = ok && c[d] >= lo[d] && c[d] < lo[d] + n[d];
		return ok;
	}
	__device__ __forceinline__ void coords(int l, int *c, int nd) const {
		for (int d = 0; d < nd; d++) {
			c[d] = lo[d] + l % n[d];
			l /= n[d];
		}
	}
};
// Box coordinates of linear index l < vol without integer division: the
// block-uniform reciprocals of the extents (box_rcp) and one float multiply
// per dimension.  (l + 0.5) / n lies at least 0.5 / n from an integer and
// the float product errs by less than 2^-12 for l < 2^11 (the boxes hold at
// most 2048 nodes, extents <= 2 kBoxReach + 4), so the quotient is exact.
struct BoxRcp {
	float r[3];
};
__device__ __forceinline__ BoxRcp box_rcp(const Box &b) {
	BoxRcp q;
#pragma unroll
	for (int d = 0; d < 3; d++) q.r[d] = 1.0f / (float)b.n[d];
	return q;
}
#ifndef PINC_PUSH_FASTDIV
#define PINC_PUSH_FASTDIV 1
#endif
__device__ __forceinline__ void box_coords(const Box &b, const BoxRcp &q, int l, int *c, int nd) {
#if !PINC_PUSH_FASTDIV
	(void)q;
	b.coords(l, c, nd);
	return;
#endif
#pragma unroll
	for (int d = 0; d < 3; d++) {
		if (d >= nd) break;
		if (d == nd - 1) {
			c[d] = b.lo[d] + l;
			break;
		}
		const int qd = (int)(((float)l + 0.5f) * q.r[d]);
		c[d] = b.lo[d] + (l - qd * b.n[d]);
		l = qd;
	}
}
// Box of the cells clo..chi grown by grow_lo/grow_hi, trimmed to at most cap
// entries: each dimension first to kBoxReach cells either side of the mean
// cell mid, then the widest one cell at a time from its side farther from mid
// (block-uniform; vol 0 if even a single cell does not fit).
#ifndef PINC_PUSH_REACH
#define PINC_PUSH_REACH 8
#endif
constexpr int kBoxReach = PINC_PUSH_REACH;
__device__ __forceinline__ Box make_box(const int *clo, const int *chi, const int *mid, int grow_lo, int grow_hi,
                                        int nd, int cap) {
	int lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
	for (int d = 0; d < nd; d++) {
		lo[d] = max(clo[d], mid[d] - kBoxReach);
		hi[d] = min(chi[d], mid[d] + kBoxReach);
		if (lo[d] > hi[d]) lo[d] = hi[d] = mid[d];
	}
	long v = 0;
#pragma unroll 1
	for (int it = 0; it < 6 * kBoxReach + 3; it++) {
		v = 1;
		int w = 0;
		for (int d = 0; d < nd; d++) {
			v *= hi[d] - lo[d] + 1 + grow_lo + grow_hi;
			if (hi[d] - lo[d] > hi[w] - lo[w]) w = d;
		}
		if (v <= cap || hi[w] == lo[w]) break;
		if (hi[w] - mid[w] >= mid[w] - lo[w]) hi[w]--;
		else lo[w]++;
	}
	Box b;
	for (int d = 0; d < 3; d++) {
		b.lo[d] = d < nd ? lo[d] - grow_lo : 0;
		b.n[d] = d < nd ? hi[d] - lo[d] + 1 + grow_lo + grow_hi : 1;
	}
	b.vol = (v <= cap && v > 0) ? (int)v : 0;
	return b;
}

// LDS counter add of 1 per active lane at ctr[idx], aggregated over the
// lanes that share an index: the two largest groups (first and last pending
// lane's index) take one atomic each, the rest add individually.  Returns the
// lane's rank (old value + rank among its group) when RET.
template <bool RET>
__device__ __forceinline__ int lds_agg_add(int *ctr, int idx, bool active) {
	const int lane = threadIdx.x & 63;
	unsigned long long pend = __ballot(active);
	int mine = 0;
#pragma unroll 1
	for (int grp = 0; grp < 2 && pend; grp++) {
		int leader = grp ? 63 - __clzll((long long)pend) : __ffsll((long long)pend) - 1;
		int li = __shfl(idx, leader, 64);
		unsigned long long m = __ballot(active && idx == li) & pend;
		pend &= ~m;
		int b = 0;
		if (lane == leader) b = atomicAdd(&ctr[li], __popcll(m));
		if (RET) {
			b = __shfl(b, leader, 64);
			if ((m >> lane) & 1ull) mine = b + __popcll(m & lanemask_lt());
		}
	}
	if ((pend >> lane) & 1ull) {
		int b = atomicAdd(&ctr[idx], 1);
		if (RET) mine = b;
	}
	return mine;
}

// sort key of integer cell coordinates (tile_key's order)
template <int ND>
__device__ __forceinline__ int tile_key_cells(const TileGeo &tg, const int *cin) {
	int c[3] = {0, 0, 0};
#pragma unroll
	for (int d = 0; d < ND; d++) c[d] = cin[d] < 0 ? 0 : (cin[d] > tg.cmax[d] ? tg.cmax[d] : cin[d]);
	return tile_key_of<ND>(tg, c);
}

// Bricks (TileGeo::bs) of a cell box: brick coordinates = clamped cell >> bs.
// A brick's cells have consecutive keys, so the sorting push reserves one
// range per brick and block from the cursor of the brick's first cell (the
// counts and the scan stay per cell; the other cells' cursors go unused).
struct BrickBox {
	int lo[3], n[3];
	int vol;
};
template <int ND>
__device__ __forceinline__ int clamp_cell(const TileGeo &tg, int d, int c) {
	return c < 0 ? 0 : (c > tg.cmax[d] ? tg.cmax[d] : c);
}
// brick box of a cell box (at most as many entries as the cell box)
template <int ND>
__device__ __forceinline__ BrickBox make_brick_box(const TileGeo &tg, const Box &b) {
	BrickBox r;
	r.vol = b.vol > 0 ? 1 : 0;
#pragma unroll
	for (int d = 0; d < 3; d++) {
		r.lo[d] = d < ND ? clamp_cell<ND>(tg, d, b.lo[d]) >> tg.bs[d] : 0;
		r.n[d] = d < ND ? (clamp_cell<ND>(tg, d, b.lo[d] + b.n[d] - 1) >> tg.bs[d]) - r.lo[d] + 1 : 1;
		r.vol *= r.n[d];
	}
	return r;
}
// Brick box of the cells within `reach` of the block's mean cell (clipped to
// its extent clo..chi), trimmed to at most cap bricks -- the widest dimension
// first, from its side farther from the mean -- but never inside `core`.
template <int ND>
__device__ __forceinline__ BrickBox wide_brick_box(const TileGeo &tg, const int *clo, const int *chi, const int *mid,
                                                   int reach, int cap, const BrickBox &core) {
	int lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0}, m[3] = {0, 0, 0}, flo[3] = {0, 0, 0}, fhi[3] = {0, 0, 0};
#pragma unroll
	for (int d = 0; d < ND; d++) {
		int l = max(clo[d], mid[d] - reach), h = min(chi[d], mid[d] + reach);
		if (l > h) l = h = mid[d];
		m[d] = clamp_cell<ND>(tg, d, mid[d]) >> tg.bs[d];
		flo[d] = core.vol ? core.lo[d] : m[d];
		fhi[d] = core.vol ? core.lo[d] + core.n[d] - 1 : m[d];
		lo[d] = min(clamp_cell<ND>(tg, d, l) >> tg.bs[d], flo[d]);
		hi[d] = max(clamp_cell<ND>(tg, d, h) >> tg.bs[d], fhi[d]);
	}
	int v = 0;
#pragma unroll 1
	for (int it = 0; it < 128; it++) {
		v = 1;
		for (int d = 0; d < ND; d++) v *= hi[d] - lo[d] + 1;
		if (v <= cap) break;
		int w = -1;
		for (int d = 0; d < ND; d++)
			if ((lo[d] < flo[d] || hi[d] > fhi[d]) && (w < 0 || hi[d] - lo[d] > hi[w] - lo[w])) w = d;
		if (w < 0) break;
		if (hi[w] > fhi[w] && (lo[w] >= flo[w] || hi[w] - m[w] >= m[w] - lo[w])) hi[w]--;
		else lo[w]++;
	}
	// block-uniform: scalar registers
	BrickBox b;
#pragma unroll
	for (int d = 0; d < 3; d++) {
		b.lo[d] = __builtin_amdgcn_readfirstlane(lo[d]);
		b.n[d] = __builtin_amdgcn_readfirstlane(hi[d] - lo[d] + 1);
	}
	b.vol = __builtin_amdgcn_readfirstlane(v <= cap ? v : 0);
	return b;
}
// index in the brick box of the brick holding cell c, or -1 outside it
template <int ND>
__device__ __forceinline__ int brick_inside(const TileGeo &tg, const BrickBox &bb, const int *c) {
	int l = 0, s = 1;
	bool in = bb.vol > 0;
#pragma unroll
	for (int d = 0; d < ND; d++) {
		const int r = (clamp_cell<ND>(tg, d, c[d]) >> tg.bs[d]) - bb.lo[d];
		in &= (unsigned)r < (unsigned)bb.n[d];
		l += mul24(r, s);
		s *= bb.n[d];
	}
	return in ? l : -1;
}
// key of the first cell of the brick holding cell c
template <int ND>
__device__ __forceinline__ int brick_first_key(const TileGeo &tg, const int *c) {
	int f[3] = {0, 0, 0};
#pragma unroll
	for (int d = 0; d < ND; d++) f[d] = (clamp_cell<ND>(tg, d, c[d]) >> tg.bs[d]) << tg.bs[d];
	return tile_key_cells<ND>(tg, f);
}
// key of the first cell of brick l of a brick box
template <int ND>
__device__ __forceinline__ int brick_key(const TileGeo &tg, const BrickBox &bb, int l) {
	int c[3] = {0, 0, 0};
#pragma unroll
	for (int d = 0; d < ND; d++) {
		c[d] = (bb.lo[d] + l % bb.n[d]) << tg.bs[d];
		l /= bb.n[d];
	}
	return tile_key_cells<ND>(tg, c);
}

typedef double dvec2 __attribute__((ext_vector_type(2)));

// chunk of push block b of nb.  PINC_PUSH_XCD: consecutive chunks (the same
// cell tiles after a sort: shared E nodes and rho atomics) on one XCD's L2.
// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md,
// workgroup dispatch), so block b runs on XCD b % 8; the map is a bijection
// for any grid size and only a placement hint, never needed for
// correctness.  (Host and device: the push trace attributes chunks to XCDs
// with it, pinc_hip_push_xcd_of_chunk.)
__host__ __device__ __forceinline__ unsigned push_chunk_of(unsigned nb, unsigned b) {
#if PINC_PUSH_XCD == 2
	// pieces of PINC_PUSH_XCD_PIECE consecutive chunks dealt round-robin over
	// the XCDs (the tail beyond whole rounds in order): every XCD gets pieces
	// from every part of the array, e.g. both z faces' tiles, where wrapped
	// particles make blocks slower
	constexpr unsigned P = PINC_PUSH_XCD_PIECE;
	const unsigned F = nb / (8u * P) * (8u * P);
	if (b >= F) return b;
	const unsigned x = b & 7u, y = b >> 3;
	return ((y / P) * 8u + x) * P + (y % P);
#elif PINC_PUSH_XCD
	const unsigned x = b & 7u, y = b >> 3;
	const unsigned q = nb >> 3, r = nb & 7u;
	return x * q + (x < r ? x : r) + y;
#else
	(void)nb;
	return b;
#endif
}

// OBJ: the object test of the fused collection (separate instances, so the
// plain push carries none of its code)
template <int ND, bool V3D, bool KICK, bool SORT, bool OBJ = false>
__global__ __launch_bounds__(kPushThreads) __attribute__((amdgpu_waves_per_eu(PINC_PUSH_WPE))) void k_push(PushArgs a) {
	constexpr int NC = 1 << ND;
	constexpr int NW = kPushThreads / 64;
	// the sorting push keeps its LDS at 40 KB (4 blocks per CU): fewer copies
	constexpr int RL = SORT ? 1024 : kRhoLds;
	__shared__ double rhoL[RL];
	// staged E box: 3-D (E_x, E_y) pairs at eL[2t] (one ds_read_b128 per
	// corner) and E_z at eL[2 cap + t], else value-major
	constexpr int EC = SORT ? kEBoxCapSort : kEBoxCapPlain;  // E box capacity (nodes)
	constexpr int RC = SORT ? kRhoBoxCap : RL;              // charge box capacity (nodes)
	constexpr int kEL = KICK ? EC * ND : 1;
	__shared__ __attribute__((aligned(16))) double eLs[kEL];
	double *const eL = eLs;
	__shared__ int cntOut[kOutCellCap];
	__shared__ int red[3 * 3 * NW];
	__shared__ int cbox[9];
	__shared__ double kered[NW];
	__shared__ int wcnt[NW];
	__shared__ int wmov[NW];
	// sorting push, per item: its rank code (phase C) and its flag (phase D)
	__shared__ int rlL[SORT ? kPushChunk : 1];
	// sorting push with PINC_SORT_CELLRANK: counters, then exclusive offsets,
	// of (brick, cell in brick)
	__shared__ int ccL[(SORT && PINC_SORT_CELLRANK) ? kCellRankBricks * 16 : 1];
	__shared__ unsigned char stageF[SORT ? kPushChunk : 1];
	const Geo32 G = make_geo32(a.g);
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	// chunk of this block (push_chunk_of: XCD-aware placement)
	const unsigned chunk = push_chunk_of(gridDim.x, blockIdx.x);
	const long base = (long)chunk * kPushChunk;
	// item k of a thread: particles in lane-contiguous pairs (16-B loads and
	// stores, 1 KiB per wave instruction), pair k/2 of the thread
#if PINC_PUSH_CONSEC && PINC_PUSH_XCH == 2
	// the kPushItems particles of a thread are consecutive, so a thread's
	// particles mostly share a cell and their charge is summed in the thread
	// before the LDS adds; rows of 16 lanes swap halves so that full blocks
	// load and store contiguously (PINC_PUSH_XCH): row r of a wave holds the
	// 64 consecutive particles at {0, 128, 64, 192}[r], lane i of it those
	// at 4i of them
	static_assert(kPushItems == 4 && kPushThreads % 64 == 0, "lane exchange: four items per thread");
	auto item = [&](int k) -> long {
		return base + (long)(wv * 256 + ((lane >> 4) & 1) * 128 + (lane >> 5) * 64 + (lane & 15) * 4 + k);
	};
#elif PINC_PUSH_CONSEC && PINC_PUSH_XCH
	// the kPushItems particles of a thread are consecutive, so a thread's
	// particles mostly share a cell and their charge is summed in the thread
	// before the LDS adds; lane pairs swap halves so that full blocks load
	// and store contiguously (PINC_PUSH_XCH)
	static_assert(kPushItems == 4 && kPushThreads % 64 == 0, "lane exchange: four items per thread");
	auto item = [&](int k) -> long {
		return base + (long)(wv * 256 + (lane & 1) * 128 + (lane >> 1) * 4 + k);
	};
#elif PINC_PUSH_CONSEC
	// the kPushItems particles of a thread are consecutive (two 16-B loads per
	// array and thread: a wave instruction covers every other 16 B of 2 KB,
	// the next one the rest, through L2), so a thread's particles mostly share
	// a cell and their charge is summed in the thread before the LDS adds
	auto item = [&](int k) -> long { return base + (long)(kPushItems * threadIdx.x + k); };
#else
	auto item = [&](int k) -> long { return base + (long)((k >> 1) * (2 * kPushThreads) + 2 * threadIdx.x + (k & 1)); };
#endif
	// pairs are 16-B aligned when every species array is (the species
	// offset iStart is even); otherwise one 8-B access per particle
	bool al = true;
#pragma unroll
	for (int d = 0; d < ND; d++)
		al = al && !((reinterpret_cast<unsigned long>(a.xi[d]) | reinterpret_cast<unsigned long>(a.vi[d]) |
		              reinterpret_cast<unsigned long>(a.xo[d]) | reinterpret_cast<unsigned long>(a.vo[d])) & 15);

	unsigned long long tsub = 0;  // (trace mode: thread 0's last timestamp)
	// (PINC_PUSH_PRIO: a block's waves issue their particle loads at raised
	// wave priority, so the memory pipe is fed before older blocks' compute)
	if (PINC_PUSH_PRIO > 0) __builtin_amdgcn_s_setprio(PINC_PUSH_PRIO);
	PUSH_TS(0);
	// ---- phase A: load every item, cell box of the input positions (periodic
	// images nearest to the cell of the block's first item)
	// (loaded first, converted after the item loads are issued: the oldest
	// load in flight, so its wait does not hold back the items')
	double xref[3] = {1.0, 1.0, 1.0};
	if (base < a.n) {
#pragma unroll
		for (int d = 0; d < ND; d++) xref[d] = a.xi[d][base];
	}
	double p[kPushItems][ND], vv[kPushItems][ND];
	unsigned valid = 0;
	static_assert(kPushItems % 2 == 0, "items come in pairs");
#if PINC_PUSH_CONSEC && PINC_PUSH_XCH
	// a full block of aligned arrays: two contiguous 16-B loads per array and
	// thread (wave pairs lane and 64 + lane), then the odd lane's first pair
	// and the even lane's second pair change places (quad_perm [1,0,3,2])
	const bool full = al && base + kPushChunk <= a.n;
	const bool odd = lane & 1;
	auto swap_adj = [](dvec2 v) -> dvec2 { return dvec2{dpp<kDppQuadXor1>(v.x), dpp<kDppQuadXor1>(v.y)}; };
	// (XCH 2) lane l loads pair pi(l) and 64 + pi(l) of the wave's 128: rows 0
	// and 1 (2 and 3) interleave pairs 0..31 (32..63) even/odd, so the row
	// swap (v_permlane16_swap: odd rows of the first <-> even rows of the
	// second) leaves each lane two consecutive pairs; every wave instruction
	// still covers one contiguous 1 KB
	auto pi_lane = [](int l) { return ((l >> 5) << 5) + 2 * (l & 15) + ((l >> 4) & 1); };
	auto rowswap = [](dvec2 &u, dvec2 &w) {
		typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
		u32x4 A = __builtin_bit_cast(u32x4, u), B = __builtin_bit_cast(u32x4, w);
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const auto r = __builtin_amdgcn_permlane16_swap(A[i], B[i], false, false);
			A[i] = r[0];
			B[i] = r[1];
		}
		u = __builtin_bit_cast(dvec2, A);
		w = __builtin_bit_cast(dvec2, B);
	};
	(void)pi_lane;
	(void)rowswap;
	if (full && PINC_PUSH_XCH == 2) {
		valid = (1u << kPushItems) - 1;
		const long q0 = base + wv * 256 + 2 * pi_lane(lane);
		auto ld = [](const double *ptr) -> dvec2 {
			if (PINC_PUSH_XCH_NT & 1) return __builtin_nontemporal_load(reinterpret_cast<const dvec2 *>(ptr));
			return *reinterpret_cast<const dvec2 *>(ptr);
		};
#pragma unroll
		for (int d = 0; d < ND; d++) {
			dvec2 x0 = ld(a.xi[d] + q0);
			dvec2 x1 = ld(a.xi[d] + q0 + 128);
			dvec2 v0 = ld(a.vi[d] + q0);
			dvec2 v1 = ld(a.vi[d] + q0 + 128);
			rowswap(x0, x1);
			rowswap(v0, v1);
			p[0][d] = x0.x;
			p[1][d] = x0.y;
			p[2][d] = x1.x;
			p[3][d] = x1.y;
			vv[0][d] = v0.x;
			vv[1][d] = v0.y;
			vv[2][d] = v1.x;
			vv[3][d] = v1.y;
		}
	} else if (full) {
		valid = (1u << kPushItems) - 1;
		const long q0 = base + wv * 256 + 2 * lane;  // the wave's pair `lane`; pair 64 + lane 128 later
#pragma unroll
		for (int d = 0; d < ND; d++) {
			const dvec2 x0 = *reinterpret_cast<const dvec2 *>(a.xi[d] + q0);
			const dvec2 x1 = *reinterpret_cast<const dvec2 *>(a.xi[d] + q0 + 128);
			const dvec2 v0 = *reinterpret_cast<const dvec2 *>(a.vi[d] + q0);
			const dvec2 v1 = *reinterpret_cast<const dvec2 *>(a.vi[d] + q0 + 128);
			const dvec2 xr = swap_adj(odd ? x0 : x1), vr = swap_adj(odd ? v0 : v1);
			const dvec2 xa = odd ? xr : x0, xb = odd ? x1 : xr;
			const dvec2 va = odd ? vr : v0, vb = odd ? v1 : vr;
			p[0][d] = xa.x;
			p[1][d] = xa.y;
			p[2][d] = xb.x;
			p[3][d] = xb.y;
			vv[0][d] = va.x;
			vv[1][d] = va.y;
			vv[2][d] = vb.x;
			vv[3][d] = vb.y;
		}
	} else
#endif
#pragma unroll
	for (int k = 0; k < kPushItems; k += 2) {
		const long i = item(k);
		const bool ok0 = i < a.n, ok1 = i + 1 < a.n;
		valid |= ((unsigned)ok0 | (unsigned)ok1 << 1) << k;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			if (ok1 && al) {
				// streamed once per step (far beyond L2/MALL): non-temporal
#if PINC_PUSH_CONSEC || !PINC_PUSH_NT
				const dvec2 x = *reinterpret_cast<const dvec2 *>(a.xi[d] + i);
				const dvec2 v = *reinterpret_cast<const dvec2 *>(a.vi[d] + i);
#else
				const dvec2 x = __builtin_nontemporal_load(reinterpret_cast<const dvec2 *>(a.xi[d] + i));
				const dvec2 v = __builtin_nontemporal_load(reinterpret_cast<const dvec2 *>(a.vi[d] + i));
#endif
				p[k][d] = x.x;
				p[k + 1][d] = x.y;
				vv[k][d] = v.x;
				vv[k + 1][d] = v.y;
			} else {
				p[k][d] = ok0 ? a.xi[d][i] : 1.0;
				vv[k][d] = ok0 ? a.vi[d][i] : 0.0;
				p[k + 1][d] = ok1 ? a.xi[d][i + 1] : 1.0;
				vv[k + 1][d] = ok1 ? a.vi[d][i + 1] : 0.0;
			}
		}
	}
	// (negative: the loads at priority 0, the rest of the block at -PRIO)
	if (PINC_PUSH_PRIO != 0) __builtin_amdgcn_s_setprio(PINC_PUSH_PRIO > 0 ? 0 : -PINC_PUSH_PRIO);
	int cref[3] = {0, 0, 0};
#pragma unroll
	for (int d = 0; d < ND; d++) cref[d] = __builtin_amdgcn_readfirstlane((int)xref[d]);
	// main.c's double fold (literal loop): a deposit on a slab ghost plane
	// counts twice and literal_ghost_weights adds that weight at the cell's
	// own planes, so the slab dimension keeps its unmapped cells there (an
	// image would move weight between ghost plane 0 and true plane T, which
	// one fold treats alike and two do not)
#ifndef PINC_LITERAL_SLAB_IMAGES
	const int imgMask = a.g.literal ? (a.wrapMask & ~(1 << G.slab)) : a.wrapMask;
#else
	const int imgMask = a.wrapMask;  // (variant build: the round-4 mapping, for the regression test)
#endif
	const Images img = make_images(G, imgMask, cref, ND);
	// cell range (and sum) of the block's items, in raw cells or in the
	// images nearest the reference cell
	auto cell_box = [&](bool withImg) {
		int lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN}, sm[3] = {0, 0, 0};
#pragma unroll
		for (int k = 0; k < kPushItems; k += 2) {
#pragma unroll
			for (int d = 0; d < ND; d++) {
#pragma unroll
				for (int h = 0; h < 2; h++) {
					if ((valid >> (k + h)) & 1u) {
						const int c = withImg ? img(d, (int)p[k + h][d]) : (int)p[k + h][d];
						lo[d] = min(lo[d], c);
						hi[d] = max(hi[d], c);
						sm[d] += c;
					}
				}
			}
		}
#pragma unroll
		for (int d = 0; d < ND; d++) {
			int x = wave_min_i(lo[d]), y = wave_max_i(hi[d]), z = wave_sum_i(sm[d]);
			if (lane == 0) {
				red[(3 * d) * NW + wv] = x;
				red[(3 * d + 1) * NW + wv] = y;
				red[(3 * d + 2) * NW + wv] = z;
			}
		}
		__syncthreads();
		if (threadIdx.x < ND) {
			int d = threadIdx.x, x = INT32_MAX, y = INT32_MIN, z = 0;
			for (int w = 0; w < NW; w++) {
				x = min(x, red[(3 * d) * NW + w]);
				y = max(y, red[(3 * d + 1) * NW + w]);
				z += red[(3 * d + 2) * NW + w];
			}
			const int nv = (int)min((long)kPushChunk, a.n - base);
			cbox[d] = x;
			cbox[3 + d] = y;
			cbox[6 + d] = nv > 0 ? z / nv : 0;
		}
		__syncthreads();
	};
#if PINC_PUSH_IMG_GATE
	// The images differ from the raw cells only for a block whose items
	// straddle a periodic boundary: with every raw cell within T/2 - 2 of the
	// reference cell, the pre-move cells and the post-move cells of the
	// particles that stay in place (one cell of motion) all lie strictly
	// between the images' bounds, so img() is the identity there.  Such
	// blocks (nearly all) skip the per-item image arithmetic in the box, the
	// kick and the deposit; a particle that wrapped in place lands outside
	// the charge box and adds its weights through memory (the same nodes, a
	// different summation order).  The others take the raw box first, then
	// the images' box.
	cell_box(false);
	bool useImg = false;
#pragma unroll
	for (int d = 0; d < ND; d++) {
		const int x = __builtin_amdgcn_readfirstlane(cbox[d]), y = __builtin_amdgcn_readfirstlane(cbox[3 + d]);
		useImg |= x <= y && (img.lo[d] != INT32_MIN || img.hi[d] != INT32_MAX) &&
		          (cref[d] - x > G.T[d] / 2 - 2 || y - cref[d] > G.T[d] / 2 - 2);
	}
	if (useImg) cell_box(true);
#else
	const bool useImg = true;
	cell_box(true);
#endif
	int clo[3] = {0, 0, 0}, chi[3] = {0, 0, 0}, cmid[3] = {0, 0, 0};
#pragma unroll
	for (int d = 0; d < ND; d++) {
		// block-uniform: scalar registers, so the boxes cost no VGPRs
		clo[d] = __builtin_amdgcn_readfirstlane(cbox[d]);
		chi[d] = __builtin_amdgcn_readfirstlane(cbox[3 + d]);
		cmid[d] = __builtin_amdgcn_readfirstlane(cbox[6 + d]);
	}
	const bool empty = clo[0] > chi[0];
	// E nodes of the input cells; charge nodes and cells after a move of at
	// most one cell (|v| <= maxVel <= 1).  Each box is trimmed around the
	// block's mean cell to its LDS capacity; the items outside it (far movers,
	// wrapped particles) take the global path.
	const Box eB = (KICK && !empty) ? make_box(clo, chi, cmid, 0, 1, ND, EC) : Box{{0, 0, 0}, {1, 1, 1}, 0};
	const Box rB = !empty ? make_box(clo, chi, cmid, 1, 2, ND, RC) : Box{{0, 0, 0}, {1, 1, 1}, 0};
	// (the sorting push's cell box: the core of its brick box ib below)
	const int ahead = PINC_SORT_AHEAD ? 1 : 0;  // (sort cells: input cells +-1, sort_cell)
	const Box iB = (SORT && !empty) ? make_box(clo, chi, cmid, ahead, ahead, ND, kInCellCap) : Box{{0, 0, 0}, {1, 1, 1}, 0};
	// the sorting push reserves per brick from the cursor of the brick's
	// first cell, so the counting push counts per brick (at its first key):
	// a block's output falls into a few bricks.  Only the brick counters live
	// in LDS, so the cell box they cover may be 16 times their number; a
	// brick box beyond the counters (far movers) counts in memory.
	const Box oB = (a.cntNext && !empty) ? make_box(clo, chi, cmid, 1 + ahead, 1 + ahead, ND, 16 * kOutCellCap)
	                                     : Box{{0, 0, 0}, {1, 1, 1}, 0};
	BrickBox obb = (a.cntNext && !empty) ? make_brick_box<ND>(a.tg, oB) : BrickBox{{0, 0, 0}, {1, 1, 1}, 0};
	if (obb.vol > kOutCellCap) obb.vol = 0;
	// sorting push: the items inside the wide brick box ib are ranked by
	// brick (one run of each brick per block); only items outside it take a
	// global slot one by one.  The brick counters live in cntOut, which a
	// sorting push does not use (it never counts).
	int slo[3] = {0, 0, 0}, shi[3] = {0, 0, 0};
#pragma unroll
	for (int d = 0; d < ND; d++) {
		slo[d] = clo[d] - ahead;
		shi[d] = chi[d] + ahead;
	}
	const BrickBox ib = (SORT && !empty)
	                        ? wide_brick_box<ND>(a.tg, slo, shi, cmid, 8, kInCellCap, make_brick_box<ND>(a.tg, iB))
	                        : BrickBox{{0, 0, 0}, {1, 1, 1}, 0};
	static_assert(kOutCellCap >= 2 * kInCellCap, "brick counters in cntOut");
	int *const bCnt = cntOut, *const bBase = cntOut + kInCellCap;

	PUSH_TS(1);
	// ---- phase B: LDS setup (zero the accumulators, stage E)
	// copies of the charge box (PINC_PUSH_COPIES): odd stride, so that the
	// copies of a node fall in different LDS banks
	const int rStride = rB.vol | 1;
	int nCopy = 1;
	while (nCopy < PINC_PUSH_COPIES && 2 * nCopy * rStride <= RL) nCopy *= 2;
	const int myCopy = (lane & (nCopy - 1)) * rStride;
	for (int t = threadIdx.x; t < (PINC_PUSH_COPIES ? nCopy * rStride : rB.vol); t += kPushThreads) rhoL[t] = 0.0;
	for (int t = threadIdx.x; t < (SORT ? kInCellCap : obb.vol); t += kPushThreads) cntOut[t] = 0;
	// (cell ranking: block-uniform; bricks of at most 16 cells)
	const int brickCellBits = a.tg.bs[0] + a.tg.bs[1] + a.tg.bs[2];
	const bool cellRank = SORT && PINC_SORT_CELLRANK && ib.vol <= kCellRankBricks && brickCellBits <= 4;
	if (cellRank)
		for (int t = threadIdx.x; t < ib.vol * 16; t += kPushThreads) ccL[t] = 0;
	if (KICK && !(PINC_PUSH_SKIP & 2)) {
		const BoxRcp eq = box_rcp(eB);
		for (int t = threadIdx.x; t < eB.vol; t += kPushThreads) {
			int c[3] = {0, 0, 0};
			box_coords(eB, eq, t, c, ND);
			int off = 0;
#pragma unroll
			for (int d = 0; d < ND; d++) {
				int o0, o1;
				node_pair(G, d, c[d], o0, o1);
				off += o0;
			}
			const double *ep = a.Es + (unsigned)(off * ND);
			if constexpr (ND == 3) {
				eL[2 * t] = ep[0];
				eL[2 * t + 1] = ep[1];
				eL[2 * EC + t] = ep[2];
			} else {
#pragma unroll
				for (int q = 0; q < ND; q++) eL[t * ND + q] = ep[q];
			}
		}
	}
	__syncthreads();

	int resBase = 0;  // sorting push: this thread's brick reservation
	PUSH_TS(2);
	// ---- phase C (sorted output): rank of every item inside its brick's run,
	// and one global reservation per brick of the block.  Per item, in LDS
	// (the sort push is tight on VGPRs): rank << 8 | brick of ib, or ~global
	// slot for an item outside ib.  A brick's run holds its cells in the order
	// the items reach the counter: a wave instruction's same-cell lanes stay
	// together, so a thread's consecutive output particles mostly share a cell
	// (round 4: ranking by cell inside each brick first cost a pass and two
	// barriers; C4 electron sorting push 33.9 -> 32.0 ms, the plain pushes
	// after it +1 %).
	if (SORT) {
		static_assert(kInCellCap <= 256 && kPushChunk <= (1 << 23), "rank/brick packing");
		static_assert(kCellRankBricks <= 64 && kPushChunk <= (1 << 20), "rank/brick/cell packing");
		int no = 0;  // (trace: items outside ib)
#pragma unroll
		for (int k = 0; k < kPushItems; k++) {
			int c[3] = {0, 0, 0};
#pragma unroll
			for (int d = 0; d < ND; d++) c[d] = sort_cell(p[k][d], vv[k][d]);
			const bool ok = (valid >> k) & 1u;
			const int lb = ok ? brick_inside<ND>(a.tg, ib, c) : -1;
			// plain LDS atomics: a wave's lanes share a few bricks (same-address
			// conflicts), cheaper than aggregating the groups with ballots and
			// shuffles (C4 electron sorting push 36.2 -> 33.5 ms)
			int rank = 0, rl = -1;
			if (cellRank) {
				// the cell's index inside its brick, x fastest (clamped as brick_inside)
				int ci = 0, sh = 0;
#pragma unroll
				for (int d = 0; d < ND; d++) {
					ci |= (clamp_cell<ND>(a.tg, d, c[d]) & ((1 << a.tg.bs[d]) - 1)) << sh;
					sh += a.tg.bs[d];
				}
				rank = lb >= 0 ? atomicAdd(&ccL[lb * 16 + ci], 1) : 0;
				rl = rank << 10 | lb << 4 | ci;
			} else {
				rank = lb >= 0 ? atomicAdd(&bCnt[lb], 1) : 0;
				rl = rank << 8 | lb;
			}
			const bool out = ok && lb < 0;
			const int g = agg_add(a.cursor, out ? brick_first_key<ND>(a.tg, c) : 0, out);
			rl = lb >= 0 ? rl : (ok ? ~g : -1);
			rlL[k * kPushThreads + threadIdx.x] = rl;  // (stored at once: no item's rank stays live)
			no += rl < 0 && ok;
		}
		if (a.diag) {
			no = wave_sum_i(no);
			if (lane == 0 && no) atomicAdd(&a.diag[0], (unsigned long long)no);
		}
		__syncthreads();
		PUSH_SUB(4);
		static_assert(kInCellCap <= kPushThreads, "one reservation per thread");
		// one global reservation per brick of ib, one range of its first
		// cell's cursor
		int bm = 0;
		if (cellRank) {
			// each brick's cell counters to exclusive offsets inside its run
			if ((int)threadIdx.x < ib.vol) {
#pragma unroll
				for (int q = 0; q < 16; q++) {
					const int v = ccL[threadIdx.x * 16 + q];
					ccL[threadIdx.x * 16 + q] = bm;
					bm += v;
				}
			}
		} else {
			bm = (int)threadIdx.x < ib.vol ? bCnt[threadIdx.x] : 0;
		}
		// the global reservation's result is first needed by the stores after
		// the kick: its round trip overlaps the kick (resBase, one VGPR)
		if (bm) resBase = atomicAdd(&a.cursor[brick_key<ND>(a.tg, ib, threadIdx.x)], bm);
	}

	PUSH_TS(3);
	// ---- phase D: kick, drift, classify (unsorted: store)
	// value offsets of the 2^ND corners in the staged E box (block-uniform)
	int eoffs[NC];
#pragma unroll
	for (int c = 0; c < NC; c++) {
		int o = 0, st = 1;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			o += ((c >> d) & 1) ? st : 0;
			st *= eB.n[d];
		}
		eoffs[c] = ND == 3 ? o : o * ND;
	}
	double ke = 0.0;
	int cnt = 0, bad = 0;
	unsigned dep = 0;
#if PINC_PUSH_LEAN
	bool thrInFrame = true;
#pragma unroll
	for (int d = 0; d < ND; d++) thrInFrame &= a.thr.lo[d] >= 0.0 && a.thr.up[d] <= a.thr.hi[d];
#endif
	// positions (and velocities if kicked or moved) of items k, k + 1
	const bool wvel = KICK || a.vo[0] != a.vi[0];
	auto store_pair = [&](int k) {
		const long i = item(k);
		const bool ok0 = (valid >> k) & 1u, ok1 = (valid >> (k + 1)) & 1u;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			if (ok1 && al) {
#if PINC_PUSH_CONSEC || !PINC_PUSH_NT
				*reinterpret_cast<dvec2 *>(a.xo[d] + i) = dvec2{p[k][d], p[k + 1][d]};
				if (wvel) *reinterpret_cast<dvec2 *>(a.vo[d] + i) = dvec2{vv[k][d], vv[k + 1][d]};
#else
				__builtin_nontemporal_store(dvec2{p[k][d], p[k + 1][d]}, reinterpret_cast<dvec2 *>(a.xo[d] + i));
				if (wvel)
					__builtin_nontemporal_store(dvec2{vv[k][d], vv[k + 1][d]}, reinterpret_cast<dvec2 *>(a.vo[d] + i));
#endif
			} else {
				if (ok0) a.xo[d][i] = p[k][d];
				if (ok0 && wvel) a.vo[d][i] = vv[k][d];
				if (ok1) a.xo[d][i + 1] = p[k + 1][d];
				if (ok1 && wvel) a.vo[d][i + 1] = vv[k + 1][d];
			}
		}
	};
#pragma unroll
	for (int k = 0; k < kPushItems; k++) {
		if (!((valid >> k) & 1u)) continue;
		const long i = item(k);
		if (KICK) {
			double dec[3], comp[3];
			int j[3] = {0, 0, 0}, jc[3] = {0, 0, 0};
#pragma unroll
			for (int d = 0; d < ND; d++) {
				j[d] = (int)p[k][d];
				jc[d] = j[d];
				dec[d] = p[k][d] - j[d];
				comp[d] = 1 - dec[d];
			}
			if (useImg) {
#pragma unroll
				for (int d = 0; d < ND; d++) jc[d] = img(d, j[d]);
			}
			// all 2^ND corners in the staged box: one unsigned compare per
			// dimension, evaluated without short-circuit branches
			bool inE = eB.vol > 0;
#pragma unroll
			for (int d = 0; d < ND; d++) inE &= (unsigned)(jc[d] - eB.lo[d]) < (unsigned)(eB.n[d] - 1);
			if (a.diag) {  // (trace: [1] += particles that gather E from memory, [3] += those of them
				           // more than a quarter of the grid from the box: periodic wraps)
				const int ng = __popcll(__ballot(!inE));
				bool far = false;
#pragma unroll
				for (int d = 0; d < ND; d++) far |= abs(jc[d] - (eB.lo[d] + eB.n[d] / 2)) > G.T[d] / 4;
				const int nf = __popcll(__ballot(!inE && far));
				if (lane == 0 && ng) atomicAdd(&a.diag[1], (unsigned long long)ng);
				if (lane == 0 && nf) atomicAdd(&a.diag[3], (unsigned long long)nf);
			}
			double dv[ND];
			if constexpr (V3D) {
				// puInterp3D1 (pusher.c:1116-1120), corner c = x + 2y + 4z, one
				// component at a time (E_x and E_y from one 16-B LDS read per
				// corner, then E_z): 16 corner values live instead of 24
				const double x = dec[0], y = dec[1], z = dec[2];
				const double xc = comp[0], yc = comp[1], zc = comp[2];
				auto interp = [&](const double *f) -> double {
					return zc * (yc * (xc * f[0] + x * f[1]) + y * (xc * f[2] + x * f[3])) +
					       z * (yc * (xc * f[4] + x * f[5]) + y * (xc * f[6] + x * f[7]));
				};
				if (PINC_PUSH_SKIP & 2) {
					dv[0] = dv[1] = dv[2] = 0.0;
				} else if (inE) {
					const int ei = eB.index(jc, ND);
					double fx[NC], fy[NC];
#pragma unroll
					for (int c = 0; c < NC; c++) {
						const dvec2 xy = *reinterpret_cast<const dvec2 *>(eL + 2 * (ei + eoffs[c]));
						fx[c] = xy.x;
						fy[c] = xy.y;
					}
					dv[0] = interp(fx);
					dv[1] = interp(fy);
					__builtin_amdgcn_sched_barrier(0);
					double fz[NC];
#pragma unroll
					for (int c = 0; c < NC; c++) fz[c] = eL[2 * EC + ei + eoffs[c]];
					dv[2] = interp(fz);
				} else {
					int o[3][2];
#pragma unroll
					for (int d = 0; d < ND; d++) node_pair(G, d, j[d], o[d][0], o[d][1]);
					unsigned off[NC];
#pragma unroll
					for (int c = 0; c < NC; c++) {
						int t = 0;
#pragma unroll
						for (int d = 0; d < ND; d++) t += o[d][(c >> d) & 1];
						off[c] = (unsigned)(t * ND);
					}
#pragma unroll
					for (int q = 0; q < ND; q++) {
						double f[NC];
#pragma unroll
						for (int c = 0; c < NC; c++) f[c] = a.Es[off[c] + q];
						dv[q] = interp(f);
					}
				}
			} else {
				double e[NC][ND];
				if (PINC_PUSH_SKIP & 2) {
#pragma unroll
					for (int c = 0; c < NC; c++)
#pragma unroll
						for (int q = 0; q < ND; q++) e[c][q] = 0.0;
				} else if (inE) {
					const double *eb = eL + mul24(eB.index(jc, ND), ND);
#pragma unroll
					for (int c = 0; c < NC; c++)
#pragma unroll
						for (int q = 0; q < ND; q++) e[c][q] = eb[eoffs[c] + q];
				} else {
					int o[3][2];
#pragma unroll
					for (int d = 0; d < ND; d++) node_pair(G, d, j[d], o[d][0], o[d][1]);
#pragma unroll
					for (int c = 0; c < NC; c++) {
						int off = 0;
#pragma unroll
						for (int d = 0; d < ND; d++) off += o[d][(c >> d) & 1];
						const double *ep = a.Es + (unsigned)(off * ND);
#pragma unroll
						for (int q = 0; q < ND; q++) e[c][q] = ep[q];
					}
				}
				// puInterpND1Inner: corner by corner in the recursion order
#pragma unroll
				for (int q = 0; q < ND; q++) dv[q] = 0;
#pragma unroll
				for (int c = 0; c < (1 << (ND - 1)); c++) {
					double f = 1.0;
					int cc = 0;
#pragma unroll
					for (int d = ND - 1; d >= 1; d--) {
						int bit = (c >> (d - 1)) & 1;
						f = (bit ? dec[d] : comp[d]) * f;
						cc |= bit << d;
					}
#pragma unroll
					for (int q = 0; q < ND; q++) {
						dv[q] += comp[0] * f * e[cc][q];
						dv[q] += dec[0] * f * e[cc | 1][q];
					}
				}
			}
			double vsq = 0;
#pragma unroll
			for (int d = 0; d < ND; d++) {
				vsq += vv[k][d] * (vv[k][d] + dv[d]);
				vv[k][d] = vv[k][d] + dv[d];
			}
			ke += vsq;
		}
		// drift + pVelAssertMax (population.c:342-365)
		int chg = 0;
#if PINC_PUSH_LEAN
		int c0[3] = {0, 0, 0};  // pre-move cell (the statistic below)
#pragma unroll
		for (int d = 0; d < ND; d++) c0[d] = (int)p[k][d];
#endif
#pragma unroll
		for (int d = 0; d < ND; d++) {
			bad |= (vv[k][d] > a.maxVel);
			p[k][d] += vv[k][d];
			// cell changed (statistic for the sort schedule; recomputed, not kept)
#if PINC_PUSH_LEAN
			chg |= (int)p[k][d] != c0[d];
#else
			chg |= (int)p[k][d] != (int)(p[k][d] - vv[k][d]);
#endif
		}
		// neighbour digit per dimension, as k_move_classify
		int ne = 0;
		bool outside = false;
#if PINC_PUSH_LEAN
		int digs[3] = {1, 1, 1};
		bool leaves = false;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			digs[d] = 1 - (p[k][d] < a.thr.lo[d]) + (p[k][d] >= a.thr.up[d]);
			leaves |= digs[d] != 1;
		}
		// a particle inside [lo, up) in every dimension is inside the frame
		// when 0 <= lo and up <= hi (thrInFrame): the frame test and the
		// in-place wrap only for the few that cross a threshold
		if (leaves || !thrInFrame) {
#pragma unroll
			for (int d = 0; d < ND; d++) {
				const double q = p[k][d] - (double)(digs[d] - 1) * (a.thr.hi[d] - 1.0);
				outside |= (q < 0.0 || q > a.thr.hi[d]);
				if ((a.wrapMask >> d) & 1) {
					if (digs[d] != 1) p[k][d] = p[k][d] + (double)((1 - digs[d]) * a.thr.T[d]);
					digs[d] = 1;
				}
			}
		}
#pragma unroll
		for (int d = ND - 1; d >= 0; d--) ne = ne * 3 + digs[d];
#else
#pragma unroll
		for (int d = ND - 1; d >= 0; d--) {
			int dig = 1 - (p[k][d] < a.thr.lo[d]) + (p[k][d] >= a.thr.up[d]);
			double q = p[k][d] - (double)(dig - 1) * (a.thr.hi[d] - 1.0);
			outside |= (q < 0.0 || q > a.thr.hi[d]);
			if ((a.wrapMask >> d) & 1) {
				if (dig != 1) p[k][d] = p[k][d] + (double)((1 - dig) * a.thr.T[d]);
				dig = 1;
			}
			ne = ne * 3 + dig;
		}
#endif
		// pPosAssertInLocalFrame fails for this particle (the host stops the
		// run with msg(ERROR) before the next deposit): route it to the
		// emigrant path so that nothing indexes the grid with it
		bad |= (int)outside << 1;
		if (outside) ne = 0;
		if (OBJ && ne == a.center) {
			// oCollectObjectCharge (object.c:489-494): the cell's lower node,
			// looked up only inside the objects' bounding box (which lies in
			// the node table: 32-bit index)
			bool inBB = true;
#pragma unroll
			for (int d = 0; d < ND; d++) inBB &= (unsigned)((int)p[k][d] - a.objLo[d]) <= (unsigned)a.objExt[d];
			unsigned node = (unsigned)(int)p[k][0];
			if (ND > 1) node += (unsigned)(int)p[k][1] * (unsigned)a.objSy;
			if (ND > 2) node += (unsigned)(int)p[k][2] * (unsigned)a.objSz;
			const int id = inBB ? a.objIn[node] : 0;
			if (id) {
				ne = PINC_NE_SINK;
				atomicAdd(&a.objCount[id - 1], 1);  // rare: particles entering an object
			}
		}
		if (SORT) {
			stageF[k * kPushThreads + threadIdx.x] = (unsigned char)ne;  // by item
		}
		// (sparse: the species' flags are the centre already -- the last
		// extraction put them back -- so only the leavers' are written, 1 B
		// per particle less at one rank, where every dimension wraps in place)
		if (!SORT && (!a.flagsSparse || ne != a.center)) a.flags[i] = (unsigned char)ne;
		if (ne != a.center) {
			cnt++;
		} else {
			dep |= (1u | (unsigned)chg << 16) << k;  // bits 16+: changed cell
		}
	}
	// (all pairs after the last kick: storing each pair right after its
	// kick, to free its velocity registers, measured 20.6 -> 26.2 ms per
	// plain push at C4, profiles/r05j_push_early_store_ab.txt)
#if PINC_PUSH_CONSEC && PINC_PUSH_XCH
	if (!SORT && full && PINC_PUSH_XCH == 2) {
		// the load's row swap backwards (an involution)
		const long q0 = base + wv * 256 + 2 * pi_lane((int)(threadIdx.x & 63));
		auto put = [&](double *o, const double (*q)[ND], int d) {
			dvec2 a0{q[0][d], q[1][d]}, a1{q[2][d], q[3][d]};
			rowswap(a0, a1);
			if (PINC_PUSH_XCH_NT & 2) {
				__builtin_nontemporal_store(a0, reinterpret_cast<dvec2 *>(o + q0));
				__builtin_nontemporal_store(a1, reinterpret_cast<dvec2 *>(o + q0 + 128));
			} else {
				*reinterpret_cast<dvec2 *>(o + q0) = a0;
				*reinterpret_cast<dvec2 *>(o + q0 + 128) = a1;
			}
		};
#pragma unroll
		for (int d = 0; d < ND; d++) {
			put(a.xo[d], p, d);
			if (wvel) put(a.vo[d], vv, d);
		}
	} else if (!SORT && full) {
		// the load's exchange backwards: contiguous 16-B stores per wave
		// instruction (pair lane, then pair 64 + lane)
		const long q0 = base + wv * 256 + 2 * lane;
		auto put = [&](double *o, const double (*q)[ND], int d) {
			const dvec2 a0{q[0][d], q[1][d]}, a1{q[2][d], q[3][d]};
			const dvec2 r = swap_adj(odd ? a0 : a1);
			*reinterpret_cast<dvec2 *>(o + q0) = odd ? r : a0;
			*reinterpret_cast<dvec2 *>(o + q0 + 128) = odd ? a1 : r;
		};
#pragma unroll
		for (int d = 0; d < ND; d++) {
			put(a.xo[d], p, d);
			if (wvel) put(a.vo[d], vv, d);
		}
	} else
#endif
	if (!SORT) {
#pragma unroll
		for (int k = 0; k < kPushItems; k += 2) store_pair(k);
	}
	PUSH_TS(4);
	if (SORT) {
		// global start of each brick's run (the reservation made before the kick)
		if ((int)threadIdx.x < ib.vol) bBase[threadIdx.x] = resBase;
		__syncthreads();
		// every item straight to its slot: the lanes of a wave instruction
		// that share a brick took consecutive ranks from its LDS counter, so
		// their stores cover one contiguous range (coalesced like the plain
		// push's) and no staging through LDS is needed
#pragma unroll
		for (int k = 0; k < kPushItems; k++) {
			if (!((valid >> k) & 1u)) continue;
			const long i = item(k);
			const int r = rlL[k * kPushThreads + threadIdx.x];
			const long o = r < 0      ? (long)~r
			               : cellRank ? (long)bBase[(r >> 4) & 63] + ccL[r & 1023] + (r >> 10)
			                          : (long)bBase[r & 255] + (r >> 8);
#pragma unroll
			for (int d = 0; d < ND; d++) {
				// (nontemporal, 8 B per lane: 24.4 -> 33.5 ms per sorting push,
				// profiles/r06i_count_runs_sort_nt_ab.txt)
				a.xo[d][o] = p[k][d];
				a.vo[d][o] = vv[k][d];
			}
			const int f = stageF[k * kPushThreads + threadIdx.x];
			if (!a.flagsSparse || f != a.center) a.flags[o] = (unsigned char)f;
			if (f != a.center) atomicAdd(&a.chunkCount[o / PINC_CHUNK], 1);
		}
	}
	PUSH_TS(5);
	if (a.cntNext && PINC_PUSH_COUNT_RUNS) {
		// count the output bricks of the particles that stay (next push's
		// sort): a thread's consecutive items mostly share one, so the items in
		// the brick of its first counted item add once (plain LDS atomics)
		int l0 = -1, nm = 0;
#pragma unroll
		for (int k = 0; k < kPushItems; k++) {
			const bool mine = (dep >> k) & 1u;
			int c[3] = {0, 0, 0};
#pragma unroll
			for (int d = 0; d < ND; d++) c[d] = sort_cell(p[k][d], vv[k][d]);
			const int lb = mine ? brick_inside<ND>(a.tg, obb, c) : -1;
			if (lb >= 0 && l0 < 0) l0 = lb;
			if (lb >= 0 && lb == l0) nm++;
			else if (lb >= 0) atomicAdd(&cntOut[lb], 1);
			if (mine && lb < 0) atomicAdd(&a.cntNext[brick_first_key<ND>(a.tg, c)], 1);
		}
		if (nm) atomicAdd(&cntOut[l0], nm);
	} else if (a.cntNext) {
		// count the output bricks of the particles that stay (next push's sort)
#pragma unroll
		for (int k = 0; k < kPushItems; k++) {
			const bool mine = (dep >> k) & 1u;
			int c[3] = {0, 0, 0};
#pragma unroll
			for (int d = 0; d < ND; d++) c[d] = sort_cell(p[k][d], vv[k][d]);
			const int lb = mine ? brick_inside<ND>(a.tg, obb, c) : -1;
			// (aggregated: plain atomics here, or after the deposit, cost the
			// plain instance, which carries this code behind a runtime test,
			// 48-52 spilled VGPRs; aggregated after the deposit: same time)
			lds_agg_add<false>(cntOut, lb < 0 ? 0 : lb, lb >= 0);
			if (mine && lb < 0) atomicAdd(&a.cntNext[brick_first_key<ND>(a.tg, c)], 1);
		}
	}
	if (bad) atomicOr(a.err, bad);
	if (!SORT || a.emigTotal) {
		int wc = wave_sum_i(cnt);
		if (lane == 0) wcnt[wv] = wc;
	}
	if (a.moved) {
		int wm = wave_sum_i(__popc(dep >> 16));
		if (lane == 0) wmov[wv] = wm;
	}

	PUSH_TS(6);
	// ---- phase E: deposit of the particles that stay
	// global fallback of one corner (nodes outside the LDS box: far movers,
	// wrapped particles, a block whose box did not fit)
	auto add_corner_global = [&](const int *j, int c, double w) {
		int off = 0;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			int o0, o1;
			node_pair(G, d, j[d], o0, o1);
			off += ((c >> d) & 1) ? o1 : o0;
		}
		unsafeAtomicAdd(&a.rho[(unsigned)off], w);
	};
	// LDS offsets of the 2^ND corners relative to the cell's lower node
	// (block-uniform: scalar registers)
	int coff[NC];
#pragma unroll
	for (int c = 0; c < NC; c++) {
		int o = 0, st = 1;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			o += ((c >> d) & 1) ? st : 0;
			st *= rB.n[d];
		}
		coff[c] = o;
	}
	// LDS index of the cell's lower node if all 2^ND corners lie in the box,
	// else -1 (one test per particle instead of one per corner)
	auto box_cell = [&](const int *j) -> int {
		bool in = rB.vol > 0;
#pragma unroll
		for (int d = 0; d < ND; d++) in &= (unsigned)(j[d] - rB.lo[d]) < (unsigned)(rB.n[d] - 1);
		return in ? rB.index(j, ND) : -1;
	};
	auto add8 = [&](const int *j, int l0, const double *w) {
		if (l0 >= 0) {
			if (PINC_PUSH_COPIES) l0 += myCopy;
#pragma unroll
			for (int c = 0; c < NC; c++) atomicAdd(&rhoL[l0 + coff[c]], w[c]);
		} else {
			if (a.diag) atomicAdd(&a.diag[2], 1ull);  // (trace: [2] += runs added to memory)
#pragma unroll
			for (int c = 0; c < NC; c++) add_corner_global(j, c, w[c]);
		}
	};
	const int keyMul[3] = {1, G.T[0] + 2, (G.T[0] + 2) * (G.T[1] + 2)};  // unique cell key
	// CIC weights and cell key of item k (a particle that stays)
	auto weights = [&](int k, int *j, double *w) -> int {
		double dec[3], comp[3];
		int kk = 0;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			j[d] = (int)p[k][d];
			dec[d] = p[k][d] - j[d];
			comp[d] = 1 - dec[d];
			kk += d ? mul24(j[d], keyMul[d]) : j[d];
		}
		cic_weights<ND, V3D>(dec, comp, w);
		literal_ghost_weights<ND>(a.g, j, w);
		// the cell's periodic image nearest the block's reference cell (the
		// boxes' coordinates): a particle that wrapped deposits into the LDS
		// box at its image nodes, which the flush maps to the same storage
		// (x, y wrapped; slab ghost planes when the slab dimension wraps,
		// folded by the halo add as every ghost deposit) instead of adding
		// its eight weights to memory
		if (useImg) {
#pragma unroll
			for (int d = 0; d < ND; d++) j[d] = img(d, j[d]);
		}
		return kk;
	};
	// one wave pass: lanes sharing a cell (up to kPushGroups groups of at
	// least kPushGroupMin lanes) are summed across the wave and added once,
	// the others add their weights one by one
	auto deposit_pass = [&](bool mine, const int *j, const double *w, int key, int l0) {
		unsigned long long pend = __ballot(mine);
		unsigned long long indiv = 0;
#pragma unroll 1
		for (int grp = 0; grp < kPushGroups && pend; grp++) {
			int leader = (grp & 1) ? 63 - __clzll((long long)pend) : __ffsll((long long)pend) - 1;
			int lk = __shfl(key, leader, 64);
			unsigned long long m = __ballot(key == lk) & pend;
			pend &= ~m;
			if (__popcll(m) < kPushGroupMin) {
				indiv |= m;
				continue;
			}
			double r[8];
			const bool in = (m >> lane) & 1ull;
#pragma unroll
			for (int c = 0; c < 8; c++) r[c] = in ? w[c] : 0.0;
			double sum = wave_reduce8(r);
			const int corner = lane >> 3;
			const int ll = __shfl(l0, leader, 64);  // leader's box cell (every lane active)
			if (ll >= 0) {
				if ((lane & 7) == 0 && corner < NC) atomicAdd(&rhoL[ll + coff[corner]], sum);
			} else {
				int jl[3] = {0, 0, 0};
#pragma unroll
				for (int d = 0; d < ND; d++) jl[d] = __shfl(j[d], leader, 64);
				if ((lane & 7) == 0 && corner < NC) add_corner_global(jl, corner, sum);
			}
		}
		indiv |= pend;
		if ((indiv >> lane) & 1ull) add8(j, l0, w);
	};
	// the two particles of a lane's pair are neighbours in memory and mostly
	// share a cell: their weights are summed in the lane first, so one wave
	// pass covers the pair's 128 particles; the second particle of a pair
	// that straddles a cell adds its weights one by one
#if PINC_PUSH_CONSEC && PINC_PUSH_COPIES
	// consecutive particles of the thread: runs of one cell are summed in
	// registers and added once (8 LDS atomics per run)
	{
		int jr[3] = {0, 0, 0}, keyr = -1;
		double wr[8];
		bool open = false;
#pragma unroll
		for (int k = 0; k < ((PINC_PUSH_SKIP & 1) ? 0 : kPushItems); k++) {
			if (!((dep >> k) & 1u)) continue;
			int jk[3] = {0, 0, 0};
			double wk[8];
			const int kk = weights(k, jk, wk);
			if (open && kk == keyr) {
#pragma unroll
				for (int c = 0; c < 8; c++) wr[c] += wk[c];
			} else {
				if (open) add8(jr, box_cell(jr), wr);
				open = true;
				keyr = kk;
#pragma unroll
				for (int d = 0; d < 3; d++) jr[d] = jk[d];
#pragma unroll
				for (int c = 0; c < 8; c++) wr[c] = wk[c];
			}
		}
		if (open) add8(jr, box_cell(jr), wr);
	}
	if (false)
#endif
#pragma unroll
	for (int k = 0; k < ((PINC_PUSH_SKIP & 1) ? 0 : kPushItems); k += 2) {
		const bool m0 = (dep >> k) & 1u, m1 = (dep >> (k + 1)) & 1u;
		int j[3] = {0, 0, 0}, j1[3] = {0, 0, 0};
		double w[8], w1[8];
#pragma unroll
		for (int c = 0; c < 8; c++) w[c] = w1[c] = 0.0;
		int key = -1, key1 = -2;
		if (m0) key = weights(k, j, w);
		if (m1) key1 = weights(k + 1, j1, w1);
		const bool merge = m0 && m1 && key == key1;
		if (merge) {
#pragma unroll
			for (int c = 0; c < 8; c++) w[c] += w1[c];
		} else if (!m0 && m1) {
#pragma unroll
			for (int d = 0; d < 3; d++) j[d] = j1[d];
#pragma unroll
			for (int c = 0; c < 8; c++) w[c] = w1[c];
			key = key1;
		}
		const int l0 = (m0 || m1) ? box_cell(j) : -1;
		if (PINC_PUSH_COPIES) {
			if (m0 || m1) add8(j, l0, w);
		} else {
			deposit_pass(m0 || m1, j, w, key, l0);
		}
		if (m0 && m1 && !merge) add8(j1, box_cell(j1), w1);
	}

	if (KICK) {
#if PINC_DPP_REDUCE
		// per-wave sums with DPP (no LDS shuffles); the block barrier below
		// publishes them
		const double w = wave_sum_d(ke);
		if (lane == 0) kered[wv] = w;
#else
		double t = block_sum(ke, kered);
		if (threadIdx.x == 0) a.kePartial[chunk] = t;
#endif
	}
	__syncthreads();
#if PINC_DPP_REDUCE
	if (KICK && threadIdx.x == 0) {
		double t = 0.0;
		for (int w = 0; w < NW; w++) t += kered[w];
		a.kePartial[chunk] = t;
	}
#endif
	if ((!SORT || a.emigTotal) && threadIdx.x == 0) {
		int t = 0;
		for (int w = 0; w < NW; w++) t += wcnt[w];
		if (!SORT && t) atomicAdd(&a.chunkCount[base / PINC_CHUNK], t);  // zeroed by the caller
		if (t && a.emigTotal) atomicAdd(a.emigTotal, (unsigned long long)t);
	}
	if (a.moved && threadIdx.x == 0) {
		int t = 0;
		for (int w = 0; w < NW; w++) t += wmov[w];
		if (t) atomicAdd(a.moved, (unsigned long long)t);
	}
	if (a.spread && threadIdx.x == 0 && !empty) {
		unsigned long long v = 1;
#pragma unroll
		for (int d = 0; d < ND; d++) v *= (unsigned long long)(chi[d] - clo[d] + 1);
		atomicAdd(a.spread, v);
	}
	// flush: one global atomic per touched node / output cell
	const BoxRcp rq = box_rcp(rB);
	for (int t = threadIdx.x; t < ((PINC_PUSH_SKIP & 4) ? 0 : rB.vol); t += kPushThreads) {
		double v = rhoL[t];
		if (PINC_PUSH_COPIES)
			for (int c = 1; c < nCopy; c++) v += rhoL[c * rStride + t];
		if (v == 0.0) continue;
		int c[3] = {0, 0, 0};
		box_coords(rB, rq, t, c, ND);
		int off = 0;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			int o0, o1;
			node_pair(G, d, c[d], o0, o1);
			off += o0;
		}
		unsafeAtomicAdd(&a.rho[(unsigned)off], v);
	}
	if (a.cntNext) {
		for (int t = threadIdx.x; t < obb.vol; t += kPushThreads) {
			int m = cntOut[t];
			if (m) atomicAdd(&a.cntNext[brick_key<ND>(a.tg, obb, t)], m);
		}
	}
	// (trace: the last phase includes every wave's drain of its stores and
	// atomics)
	if (a.tstamp) {
		__builtin_amdgcn_s_waitcnt(0);
		__syncthreads();
	}
	PUSH_TS(7);
}

// rho = chain of the species accumulators with the reference's rescaling
// (gZero; per species gMul(1/q), add, gMul(q); pusher.c:512-572)
struct CombineArgs {
	const double *acc[PINC_MAX_SPECIES];
	double q[PINC_MAX_SPECIES];
	int ns;
};

__global__ void k_rho_combine(double *__restrict__ rho, CombineArgs c, long n) {
	for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
		double r = c.acc[0][i];
		for (int s = 1; s < c.ns; s++) r = (r * c.q[s - 1]) * (1.0 / c.q[s]) + c.acc[s][i];
		rho[i] = r * c.q[c.ns - 1];
	}
}

// ------------------------------------------------- order 0 (NGP) ---------
// puDistrND0 (pusher.c:640-668) and puAccND0KE (pusher.c:310-353) with
// puInterpND0 (pusher.c:1164-1180): the nearest node (int)(x + 0.5) of the
// padded local frame takes the whole particle (one unit; the caller applies
// the species' 1/q, q chain) and lends it its E.  Not on the hot path (main.c
// offers them through select; the configs use CIC): one thread per particle,
// global atomics.
template <int ND>
__global__ __launch_bounds__(kThreads) void k_deposit_ngp(const double *__restrict__ x0,
                                                          const double *__restrict__ x1,
                                                          const double *__restrict__ x2, long b0, long n,
                                                          pinc_geom_t g, double *__restrict__ rho) {
	Geo G = make_geo(g);
	const double *xs[3] = {x0, x1, x2};
	for (long i = (long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long)gridDim.x * kThreads) {
		int j[3] = {0, 0, 0};
		long off = 0;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			j[d] = (int)(xs[d][b0 + i] + 0.5);
			off += node_off(G, d, j[d]);
		}
		const double w = g.literal ? literal_node_factor<ND>(g, j) : 1.0;
		if (w != 0.0) unsafeAtomicAdd(&rho[off], w);
	}
}

template <int ND>
__global__ __launch_bounds__(kThreads) void k_accel_ngp(const double *__restrict__ x0, const double *__restrict__ x1,
                                                        const double *__restrict__ x2, double *__restrict__ v0,
                                                        double *__restrict__ v1, double *__restrict__ v2, long b0,
                                                        long n, pinc_geom_t g, const double *__restrict__ E,
                                                        double *__restrict__ kePartial) {
	__shared__ double red[kThreads / 64];
	Geo G = make_geo(g);
	const double *xs[3] = {x0, x1, x2};
	double *vs[3] = {v0, v1, v2};
	double ke = 0.0;
	// block b owns particles [b kAccChunk, (b+1) kAccChunk): the KE partials
	// have pinc_hip_accelerate's layout
	for (int k = 0; k < kAccItems; k++) {
		const long i = (long)blockIdx.x * kAccChunk + (long)k * kThreads + threadIdx.x;
		if (i >= n) break;
		long off = 0;
#pragma unroll
		for (int d = 0; d < ND; d++) off += node_off(G, d, (int)(xs[d][b0 + i] + 0.5));
		off *= ND;
		double vsq = 0.0;
#pragma unroll
		for (int d = 0; d < ND; d++) {
			const double dv = E[off + d];
			const double vv = vs[d][b0 + i];
			vsq += vv * (vv + dv);
			vs[d][b0 + i] = vv + dv;
		}
		ke += vsq;
	}
	const double t = block_sum(ke, red);
	if (threadIdx.x == 0) kePartial[blockIdx.x] = t;
}

// pVelAssertMax (population.c:342-365): a component above maxVel (signed, as
// the reference) sets bit 0 of the assert word
__global__ __launch_bounds__(kThreads) void k_vel_assert(const double *__restrict__ v0, const double *__restrict__ v1,
                                                         const double *__restrict__ v2, long b0, long n, int nd,
                                                         double maxVel, int *__restrict__ err) {
	const double *vs[3] = {v0, v1, v2};
	int bad = 0;
	for (long i = (long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long)gridDim.x * kThreads)
		for (int d = 0; d < nd; d++) bad |= vs[d][b0 + i] > maxVel;
	if (bad) atomicOr(err, 1);
}

}  // namespace

// =========================================================== C ABI ========
extern "C" long pinc_hip_push_chunk(void) { return kPushChunk; }

extern "C" int pinc_hip_push_xcd_of_chunks(long nBlocks, int *xcd) {
	for (long b = 0; b < nBlocks; b++) xcd[push_chunk_of((unsigned)nBlocks, (unsigned)b)] = (int)(b & 7);
	return 0;
}

extern "C" int pinc_hip_deposit_ngp(pinc_pop_t pop, int s, pinc_geom_t g, double *rho, void *stream) {
	long n = pop.iStop[s] - pop.iStart[s];
	if (n <= 0) return 0;
	long b0 = pop.iStart[s];
	long nb = ceil_div(n, (long)kThreads);
	if (nb > 65536) nb = 65536;
	hipStream_t st = (hipStream_t)stream;
	const double *x1 = g.nd > 1 ? pop.x[1] : nullptr, *x2 = g.nd > 2 ? pop.x[2] : nullptr;
	if (g.nd == 3)
		hipLaunchKernelGGL(k_deposit_ngp<3>, dim3(nb), dim3(kThreads), 0, st, pop.x[0], x1, x2, b0, n, g, rho);
	else if (g.nd == 2)
		hipLaunchKernelGGL(k_deposit_ngp<2>, dim3(nb), dim3(kThreads), 0, st, pop.x[0], x1, x2, b0, n, g, rho);
	else
		hipLaunchKernelGGL(k_deposit_ngp<1>, dim3(nb), dim3(kThreads), 0, st, pop.x[0], x1, x2, b0, n, g, rho);
	return check_launch("deposit (NGP)");
}

extern "C" int pinc_hip_accelerate_ngp(pinc_pop_t pop, int s, pinc_geom_t g, const double *Es, double *kePartial,
                                       int *nBlocks, void *stream) {
	long n = pop.iStop[s] - pop.iStart[s];
	*nBlocks = 0;
	if (n <= 0) return 0;
	long b0 = pop.iStart[s];
	long nb = ceil_div(n, (long)kAccChunk);
	*nBlocks = (int)nb;
	hipStream_t st = (hipStream_t)stream;
	if (g.nd == 3)
		hipLaunchKernelGGL(k_accel_ngp<3>, dim3(nb), dim3(kThreads), 0, st, pop.x[0], pop.x[1], pop.x[2], pop.v[0],
		                   pop.v[1], pop.v[2], b0, n, g, Es, kePartial);
	else if (g.nd == 2)
		hipLaunchKernelGGL(k_accel_ngp<2>, dim3(nb), dim3(kThreads), 0, st, pop.x[0], pop.x[1], nullptr, pop.v[0],
		                   pop.v[1], nullptr, b0, n, g, Es, kePartial);
	else
		hipLaunchKernelGGL(k_accel_ngp<1>, dim3(nb), dim3(kThreads), 0, st, pop.x[0], nullptr, nullptr, pop.v[0],
		                   nullptr, nullptr, b0, n, g, Es, kePartial);
	return check_launch("accelerate (NGP)");
}

extern "C" int pinc_hip_vel_assert(pinc_pop_t pop, int s, double maxVel, int *errFlag, void *stream) {
	long n = pop.iStop[s] - pop.iStart[s];
	if (n <= 0) return 0;
	long nb = ceil_div(n, (long)kThreads * 8);
	if (nb > 16384) nb = 16384;
	long b0 = pop.iStart[s];
	hipLaunchKernelGGL(k_vel_assert, dim3(nb), dim3(kThreads), 0, (hipStream_t)stream, pop.v[0],
	                   pop.nd > 1 ? pop.v[1] : nullptr, pop.nd > 2 ? pop.v[2] : nullptr, b0, n, pop.nd, maxVel,
	                   errFlag);
	return check_launch("velocity assert");
}
extern "C" int pinc_hip_move_classify(pinc_pop_t pop, int s, int doMove, const double *thr,
                                      unsigned char *flags, int *chunkCount, double maxVel,
                                      int *errFlag, int wrapMask, void *stream) {
	long n = pop.iStop[s] - pop.iStart[s];
	if (n <= 0) return 0;
	long b0 = pop.iStart[s];
	Thr t;
	int nd = pop.nd;
	for (int d = 0; d < 3; d++) {
		t.lo[d] = d < nd ? thr[d] : 0;
		t.up[d] = d < nd ? thr[nd + d] : 0;
		t.hi[d] = d < nd ? thr[2 * nd + d] : 0;
		t.T[d] = d < nd ? (int)(thr[2 * nd + d] - 1.0 + 0.5) : 1;
	}
	int center = 0;
	for (int d = 0, p = 1; d < nd; d++, p *= 3) center += p;
	dim3 grid((unsigned)ceil_div(n, PINC_CHUNK));
	hipStream_t st = (hipStream_t)stream;
#define LAUNCH_MC(ND)                                                                          \
	hipLaunchKernelGGL(k_move_classify<ND>, grid, dim3(kThreads), 0, st, pop.x[0] + b0,        \
	                   nd > 1 ? pop.x[1] + b0 : nullptr, nd > 2 ? pop.x[2] + b0 : nullptr,     \
	                   pop.v[0] + b0, nd > 1 ? pop.v[1] + b0 : nullptr,                        \
	                   nd > 2 ? pop.v[2] + b0 : nullptr, n, doMove, t, center, flags + b0,     \
	                   chunkCount, maxVel, errFlag, wrapMask)
	if (nd == 3) LAUNCH_MC(3);
	else if (nd == 2) LAUNCH_MC(2);
	else LAUNCH_MC(1);
#undef LAUNCH_MC
	return check_launch("move_classify");
}

// pinned host words for the extraction's two small reads (a read into
// pageable memory is staged and copied again on the host's wake-up path)
static int *pinned_ints() {
	static int *p = nullptr;
	if (!p && hipHostMalloc((void **)&p, 64 * sizeof(int), hipHostMallocDefault) != hipSuccess) p = nullptr;
	return p;
}

extern "C" int pinc_hip_extract(pinc_pop_t pop, int s, unsigned char *flags, int *chunkCount,
                                int center, int nNeighbors, pinc_extract_ws_t ws, long *nEmig,
                                long *neCount, void *stream) {
	(void)nNeighbors;
	hipStream_t st = (hipStream_t)stream;
	long n = pop.iStop[s] - pop.iStart[s];
	long sb = pop.iStart[s];
	*nEmig = 0;
	for (int q = 0; q < kMaxNe; q++) neCount[q] = 0;
	if (n <= 0) return 0;
	int nChunks = (int)ceil_div(n, PINC_CHUNK);
	if (nChunks <= 4096 || !ws.scanWork) {
		hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(1024), 0, st, chunkCount, ws.chunkOffset, nChunks);
	} else {
		// multi-block scan (a single workgroup takes ~0.7 ms for 5e5 chunks)
		long nsb = ceil_div(nChunks, (long)kScanBlock);
		int *bsum = ws.scanWork, *boff = ws.scanWork + nsb;
		hipLaunchKernelGGL(k_scan_sums, dim3((unsigned)nsb), dim3(kThreads), 0, st, chunkCount, (long)nChunks, bsum);
		hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(1024), 0, st, bsum, boff, (int)nsb);
		hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nsb), dim3(kThreads), 0, st, chunkCount, (long)nChunks, boff,
		                   ws.chunkOffset);
	}
	int *hp = pinned_ints();
	if (!hp) return set_error(hipErrorOutOfMemory, "extract: pinned host words");
	hipError_t e = hipMemcpyAsync(hp, ws.chunkOffset + nChunks, sizeof(int), hipMemcpyDeviceToHost, st);
	if (e != hipSuccess) return set_error(e, "extract: count readback");
	e = hipStreamSynchronize(st);
	if (e != hipSuccess) return set_error(e, "extract: sync");
	const int E = hp[0];
	*nEmig = E;
	if (E == 0) return check_launch("extract(scan)");
	if (E > ws.cap) return PINC_ERR_CAPACITY;
	hipLaunchKernelGGL(k_extract_a, dim3(nChunks), dim3(kThreads), 0, st, flags + sb, n, center,
	                   ws.chunkOffset, nChunks, ws.tail, ws.holes, ws.order, ws.scratch);
	hipLaunchKernelGGL(k_extract_b, dim3((unsigned)ceil_div(E + 1, 256)), dim3(256), 0, st,
	                   flags + sb, n, (long)E, center, ws.tail, ws.holes, ws.order, ws.scratch);
	int nb = (int)ceil_div(E, kRankChunk);
	hipLaunchKernelGGL(k_rank_hist, dim3(nb), dim3(kThreads), 0, st, flags + sb, ws.order, (long)E,
	                   ws.blockHist);
	hipLaunchKernelGGL(k_hist_scan, dim3(1), dim3(kMaxNe * 32), 0, st, ws.blockHist, nb,
	                   ws.scratch);
	hipLaunchKernelGGL(k_rank_scatter, dim3(nb), dim3(kThreads), 0, st, flags + sb, ws.order,
	                   (long)E, ws.blockHist, ws.scratch, pop, sb, ws.buf, ws.cap, ws.bufNe, center);
	hipLaunchKernelGGL(k_fill_holes, dim3((unsigned)ceil_div(E, 256)), dim3(256), 0, st, pop, sb,
	                   ws.tail, ws.holes, ws.scratch);
	static_assert(kMaxNe <= 64, "pinned words");
	e = hipMemcpyAsync(hp, ws.scratch + 64, kMaxNe * sizeof(int), hipMemcpyDeviceToHost, st);
	if (e != hipSuccess) return set_error(e, "extract: direction counts");
	e = hipStreamSynchronize(st);
	if (e != hipSuccess) return set_error(e, "extract: sync 2");
	for (int q = 0; q < kMaxNe; q++) neCount[q] = hp[q];
	return check_launch("extract");
}

extern "C" int pinc_hip_import(pinc_pop_t pop, int s, long dst, const double *buf, long cap,
                               const unsigned char *bufNe, long first, long n, const int *shiftT,
                               int shiftMask, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_import, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
	                   (hipStream_t)stream, pop, pop.iStart[s] + dst, buf, cap, bufNe, first, n,
	                   shiftT[0], shiftT[1], shiftT[2], shiftMask);
	return check_launch("import");
}

extern "C" int pinc_hip_pack(const double *buf, long cap, const unsigned char *bufNe, long first, long n,
                             int nd, double *out, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_pack, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, buf, cap,
	                   bufNe, first, n, nd, out);
	return check_launch("pack");
}

extern "C" int pinc_hip_import_rec(pinc_pop_t pop, int s, long dst, const double *rec, long n,
                                   const int *shiftT, void *stream) {
	if (n <= 0) return 0;
	hipLaunchKernelGGL(k_import_rec, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, pop,
	                   pop.iStart[s] + dst, rec, n, shiftT[0], shiftT[1], shiftT[2]);
	return check_launch("import_rec");
}

extern "C" int pinc_hip_deposit(pinc_pop_t pop, int s, pinc_geom_t g, double *rho, void *stream) {
	long n = pop.iStop[s] - pop.iStart[s];
	if (n <= 0) return 0;
	long b0 = pop.iStart[s];
	long nb = ceil_div(n + (b0 & 1L), (long)kDepChunk);
	hipStream_t st = (hipStream_t)stream;
	const double *x0 = pop.x[0];
	const double *x1 = g.nd > 1 ? pop.x[1] : nullptr;
	const double *x2 = g.nd > 2 ? pop.x[2] : nullptr;
	if (g.nd == 3)
		hipLaunchKernelGGL((k_deposit_tiled<3, true>), dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, b0, n, g, rho);
	else if (g.nd == 2)
		hipLaunchKernelGGL((k_deposit_tiled<2, false>), dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, b0, n, g, rho);
	else
		hipLaunchKernelGGL((k_deposit_tiled<1, false>), dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, b0, n, g, rho);
	return check_launch("deposit");
}

extern "C" int pinc_hip_field_chain_all(const double *E, double *Es, long n, const double *qm, const double *mq,
                                        double pre, int nSpecies, void *stream) {
	if (n > 0 && (!E || !Es || !qm || !mq)) return set_error(hipErrorInvalidValue, "field_chain_all: null array");
	if (nSpecies < 1 || nSpecies > PINC_MAX_SPECIES)
		return set_error(hipErrorInvalidValue, "field_chain_all: species count");
	if (n <= 0) return 0;
	long nb = ceil_div(n, (long)kThreads * 4);
	if (nb > 8192) nb = 8192;
	hipLaunchKernelGGL(k_field_chain_all, dim3(nb), dim3(kThreads), 0, (hipStream_t)stream, E, Es, n, qm, mq, pre,
	                   nSpecies);
	return check_launch("field chain (all species)");
}

extern "C" int pinc_hip_field_chain(const double *E, double *Es, long n, const double *qm,
                                    const double *mq, double pre, int s, void *stream) {
	if (n > 0 && (!E || !Es || !qm || !mq)) return set_error(hipErrorInvalidValue, "field_chain: null array");
	if (n <= 0) return 0;
	long nb = ceil_div(n, (long)kThreads * 4);
	if (nb > 8192) nb = 8192;
	hipLaunchKernelGGL(k_field_chain, dim3(nb), dim3(kThreads), 0, (hipStream_t)stream, E, Es, n, qm, mq, pre, s);
	return check_launch("field chain");
}

extern "C" int pinc_hip_accelerate(pinc_pop_t pop, int s, pinc_geom_t g, const double *Es,
                                   double *kePartial, int *nBlocks, void *stream) {
	long n = pop.iStop[s] - pop.iStart[s];
	*nBlocks = 0;
	if (n <= 0) return 0;
	if (!Es) return set_error(hipErrorInvalidValue, "accelerate: null E");
	long b0 = pop.iStart[s];
	long nb = ceil_div(n + (b0 & 1L), (long)kAccChunk);
	*nBlocks = (int)nb;
	hipStream_t st = (hipStream_t)stream;
	double *x0 = pop.x[0], *x1 = pop.x[1], *x2 = pop.x[2];
	double *v0 = pop.v[0], *v1 = pop.v[1], *v2 = pop.v[2];
	if (g.nd == 3)
		hipLaunchKernelGGL((k_accel<3, true, true>), dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, v0, v1, v2, b0, n,
		                   g, Es, kePartial);
	else if (g.nd == 2)
		hipLaunchKernelGGL((k_accel<2, false, true>), dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, v0, v1, v2, b0,
		                   n, g, Es, kePartial);
	else
		hipLaunchKernelGGL((k_accel<1, false, true>), dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, v0, v1, v2, b0,
		                   n, g, Es, kePartial);
	return check_launch("accelerate");
}

extern "C" int pinc_hip_boris(pinc_pop_t pop, int s, pinc_geom_t g, const double *Es, const double *T,
                              const double *S, double *kePartial, int *nBlocks, void *stream) {
	long n = pop.iStop[s] - pop.iStart[s];
	*nBlocks = 0;
	if (g.nd != 3 || pop.nd != 3) return set_error(hipErrorInvalidValue, "boris: 3-D only (puBoris3D1)");
	if (n <= 0) return 0;
	long b0 = pop.iStart[s];
	long nb = ceil_div(n + (b0 & 1L), (long)kAccChunk);
	*nBlocks = (int)nb;
	BorisRot rot;
	for (int q = 0; q < 3; q++) {
		rot.T[q] = T[q];
		rot.S[q] = S[q];
	}
	hipLaunchKernelGGL((k_accel<3, true, true, true>), dim3(nb), dim3(kThreads), 0, (hipStream_t)stream, pop.x[0],
	                   pop.x[1], pop.x[2], pop.v[0], pop.v[1], pop.v[2], b0, n, g, Es, kePartial, rot);
	return check_launch("boris");
}

extern "C" int pinc_hip_init_species(pinc_pop_t pop, int s, pinc_geom_t g, long nGlobal,
                                     double latticeStep, const int *subdomain,
                                     const int *nSubdomains, const int *offset, const double *amp,
                                     const double *mode, int perturb, int maxwell, double drift,
                                     double vth, unsigned long long seed, long *nOut,
                                     void *stream) {
	hipStream_t st = (hipStream_t)stream;
	LatticeArgs a;
	a.nd = g.nd;
	for (int d = 0; d < 3; d++) {
		a.L[d] = d < g.nd ? g.T[d] : 1;
		a.sub[d] = d < g.nd ? subdomain[d] : 0;
		a.off[d] = d < g.nd ? offset[d] : 0;
		int tsd = d < g.nd ? (g.T[d] / nSubdomains[d]) : 1;
		a.posToSub[d] = (double)1 / tsd;
		a.amp[d] = d < g.nd ? amp[d] : 0;
		a.mode[d] = d < g.nd ? mode[d] : 0;
	}
	a.l = latticeStep;
	a.perturb = perturb;
	a.maxwell = maxwell;
	a.drift = drift;
	a.vth = vth;
	a.seed = seed;
	a.species = s;
	long nChunks = ceil_div(nGlobal, PINC_CHUNK);
	int *cnt = nullptr, *off = nullptr;
	hipError_t e = hipMallocAsync((void **)&cnt, (nChunks + 1) * sizeof(int), st);
	if (e != hipSuccess) return set_error(e, "init: alloc");
	e = hipMallocAsync((void **)&off, (nChunks + 1) * sizeof(int), st);
	if (e != hipSuccess) return set_error(e, "init: alloc");
	hipLaunchKernelGGL(k_lattice_count, dim3((unsigned)nChunks), dim3(kThreads), 0, st, a, nGlobal, cnt);
	hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(1024), 0, st, cnt, off, (int)nChunks);
	int total = 0;
	e = hipMemcpyAsync(&total, off + nChunks, sizeof(int), hipMemcpyDeviceToHost, st);
	if (e == hipSuccess) e = hipStreamSynchronize(st);
	if (e != hipSuccess) return set_error(e, "init: count readback");
	long capS = pop.iStart[s + 1] - pop.iStart[s];
	if (total > capS) {
		(void)hipFreeAsync(cnt, st);
		(void)hipFreeAsync(off, st);
		return set_error(hipErrorOutOfMemory, "init: species capacity too small");
	}
	hipLaunchKernelGGL(k_lattice_write, dim3((unsigned)nChunks), dim3(kThreads), 0, st, a, nGlobal,
	                   off, pop, pop.iStart[s]);
	(void)hipFreeAsync(cnt, st);
	(void)hipFreeAsync(off, st);
	*nOut = total;
	return check_launch("init_species");
}

// PINC_SORT_BRICK: the sorting push reserves its output per brick of
// tw^(nd-1) cells (tw x tw x 1 in 3-D, one block's worth at C4's 64 ppc)
// instead of per cell: a few tens of runs per block instead of about a
// hundred short scattered ones once the input order has decayed; inside a
// brick run the block's particles stay grouped by cell.  (Tried: bricks
// ordered along the slab dimension fastest, so that consecutive bricks are
// neighbours -- the plain pushes got slower, 25 -> 31 ms per ion launch at
// C4: the concurrently running blocks then touch scattered grid rows.)
#ifndef PINC_SORT_BRICK
#define PINC_SORT_BRICK 1
#endif

static TileGeo make_tile_geo(pinc_geom_t g, int tileWidth, long *nKeys) {
	TileGeo tg;
	long nt = 1, cpt = 1;
	tg.tw = tileWidth;
	int lw = 0;
	while ((1 << lw) < tileWidth) lw++;
	const bool brick = PINC_SORT_BRICK && (1 << lw) == tileWidth;
	for (int d = 0; d < 3; d++) {
		int T = d < g.nd ? (d == g.nd - 1 ? g.nloc : g.T[d]) : 1;
		tg.cmax[d] = T + 1;
		tg.nt[d] = d < g.nd ? (T + 1) / tileWidth + 1 : 1;
		tg.bs[d] = brick && d < g.nd - 1 ? lw : 0;
		nt *= tg.nt[d];
		if (d < g.nd) cpt *= tileWidth;
	}
	*nKeys = nt * cpt;
	return tg;
}

extern "C" int pinc_hip_sort_tiles(pinc_pop_t pop, pinc_pop_t out, int s, pinc_geom_t g, int tileWidth,
                                   int *work, long workCap, long *nKeysOut, void *stream) {
	long nk = 0;
	TileGeo tg = make_tile_geo(g, tileWidth, &nk);
	long nsb = ceil_div(nk, (long)kScanBlock);
	*nKeysOut = nk;
	// work: counts[nk+1] | offsets[nk+1] | block sums[nsb] | block offsets[nsb+1]
	long need = 2 * (nk + 1) + 2 * nsb + 1;
	if (need > workCap || nk > 2147483647L) return set_error(hipErrorInvalidValue, "sort_tiles: work buffer too small");
	long n = pop.iStop[s] - pop.iStart[s];
	if (n <= 0) return 0;
	if (n > 2147483647L) return set_error(hipErrorInvalidValue, "sort_tiles: species too large for int slots");
	long b0 = pop.iStart[s];
	hipStream_t st = (hipStream_t)stream;
	int *counts = work, *offs = work + (nk + 1), *bsum = offs + (nk + 1), *boff = bsum + nsb;
	hipError_t e = hipMemsetAsync(counts, 0, (nk + 1) * sizeof(int), st);
	if (e != hipSuccess) return set_error(e, "sort_tiles: memset");
	long nb = ceil_div(n, (long)kThreads);
	if (nb > 65536L * 8) nb = 65536L * 8;
	int nd = g.nd;
	const double *x0 = pop.x[0] + b0, *x1 = nd > 1 ? pop.x[1] + b0 : nullptr, *x2 = nd > 2 ? pop.x[2] + b0 : nullptr;
	if (nd == 3) hipLaunchKernelGGL(k_sort_count<3>, dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, n, tg, counts);
	else if (nd == 2) hipLaunchKernelGGL(k_sort_count<2>, dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, n, tg, counts);
	else hipLaunchKernelGGL(k_sort_count<1>, dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, n, tg, counts);
	hipLaunchKernelGGL(k_scan_sums, dim3((unsigned)nsb), dim3(kThreads), 0, st, counts, nk, bsum);
	hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(1024), 0, st, bsum, boff, (int)nsb);
	hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nsb), dim3(kThreads), 0, st, counts, nk, boff, offs);
	if (nd == 3) hipLaunchKernelGGL(k_sort_scatter<3>, dim3(nb), dim3(kThreads), 0, st, pop, out, b0, n, tg, offs);
	else if (nd == 2) hipLaunchKernelGGL(k_sort_scatter<2>, dim3(nb), dim3(kThreads), 0, st, pop, out, b0, n, tg, offs);
	else hipLaunchKernelGGL(k_sort_scatter<1>, dim3(nb), dim3(kThreads), 0, st, pop, out, b0, n, tg, offs);
	return check_launch("sort_tiles");
}

extern "C" int pinc_hip_deposit_cells(pinc_pop_t pop, int s, pinc_geom_t g, int tileWidth, const int *offs,
                                      long nCell, double *rho, void *stream) {
	long n = pop.iStop[s] - pop.iStart[s];
	if (n <= 0) return 0;
	long nKeys = 0;
	TileGeo tg = make_tile_geo(g, tileWidth, &nKeys);
	long b0 = pop.iStart[s];
	if (nCell > n) nCell = n;
	hipStream_t st = (hipStream_t)stream;
	const double *x0 = pop.x[0] + b0;
	const double *x1 = g.nd > 1 ? pop.x[1] + b0 : nullptr;
	const double *x2 = g.nd > 2 ? pop.x[2] + b0 : nullptr;
	unsigned nb = (unsigned)ceil_div(nKeys, (long)kThreads);
	if (g.nd == 3)
		hipLaunchKernelGGL((k_deposit_cells<3, true>), dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, nCell, offs, nKeys,
		                   tg, g, rho);
	else if (g.nd == 2)
		hipLaunchKernelGGL((k_deposit_cells<2, false>), dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, nCell, offs,
		                   nKeys, tg, g, rho);
	else
		hipLaunchKernelGGL((k_deposit_cells<1, false>), dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, nCell, offs,
		                   nKeys, tg, g, rho);
	int rc = check_launch("deposit_cells");
	if (rc || nCell >= n) return rc;
	// particles appended since the sort (immigrants): generic deposit
	pinc_pop_t tail = pop;
	tail.iStart[s] = b0 + nCell;
	return pinc_hip_deposit(tail, s, g, rho, stream);
}

extern "C" int pinc_hip_push(pinc_pop_t pop, int s, pinc_geom_t g, const pinc_push_t *args, int *nBlocks,
                             void *stream) {
	long n = pop.iStop[s] - pop.iStart[s];
	*nBlocks = 0;
	if (n <= 0) return 0;
	long b0 = pop.iStart[s];
	int nd = pop.nd;
	if (nd != g.nd) return set_error(hipErrorInvalidValue, "push: population and grid dimensions differ");
	const bool sort = args->cursor != nullptr;
	if (sort && n > 2147483647L) return set_error(hipErrorInvalidValue, "push: species too large for int slots");
	long nodes = 1;
	for (int d = 0; d < nd; d++) nodes *= (d == nd - 1) ? (long)g.nloc + 2 : (long)g.T[d];
	if (nodes * nd >= 2147483647L) return set_error(hipErrorInvalidValue, "push: grid too large for 32-bit offsets");
	PushArgs a;
	for (int d = 0; d < 3; d++) {
		a.xi[d] = d < nd ? pop.x[d] + b0 : nullptr;
		a.xo[d] = d < nd ? args->xout[d] + b0 : nullptr;
		a.vi[d] = d < nd ? pop.v[d] + b0 : nullptr;
		a.vo[d] = d < nd ? args->vout[d] + b0 : nullptr;
		a.thr.lo[d] = d < nd ? args->thr[d] : 0;
		a.thr.up[d] = d < nd ? args->thr[nd + d] : 0;
		a.thr.hi[d] = d < nd ? args->thr[2 * nd + d] : 0;
		a.thr.T[d] = d < nd ? (int)(args->thr[2 * nd + d] - 1.0 + 0.5) : 1;
	}
	a.n = n;
	a.g = g;
	a.Es = args->Es;
	a.rho = args->rhoS;
	a.center = 0;
	for (int d = 0, p = 1; d < nd; d++, p *= 3) a.center += p;
	a.wrapMask = args->wrapMask;
	a.maxVel = args->maxVel;
	a.flags = args->flags + b0;
	a.chunkCount = args->chunkCount;
	a.err = args->errFlag;
	a.kePartial = args->kePartial;
	long nKeys = 0;
	a.tg = make_tile_geo(g, args->tileWidth > 0 ? args->tileWidth : 1, &nKeys);
	a.cursor = args->cursor;
	a.cntNext = args->cntNext;
	a.moved = args->moved;
	a.spread = args->spread;
	a.tstamp = args->tstamp;
	a.diag = args->diag;
	a.emigTotal = args->emigTotal;
	a.flagsSparse = args->flagsSparse;
	a.objIn = args->objInside;
	a.objSy = args->objSy;
	a.objSz = args->objSz;
	a.objN = args->objNodes;
	a.objCount = args->objCount;
	for (int d = 0; d < 3; d++) {
		a.objLo[d] = args->objLo[d];
		a.objExt[d] = args->objHi[d] - args->objLo[d];
	}
	if (a.objIn && !a.objCount) return set_error(hipErrorInvalidValue, "push: objInside without objCount");
	if (a.objIn && (nd != 3 || a.objN > 2147483647L)) return set_error(hipErrorInvalidValue, "push: objects are 3-D");
	for (int d = 0; a.objIn && d < 3; d++)
		if (a.objExt[d] >= 0 && (a.objLo[d] < 0 || (long)a.objLo[d] + a.objExt[d] >= (d == 0 ? a.objSy : d == 1 ? a.objSz / a.objSy
		                                                                                             : a.objN / a.objSz)))
			return set_error(hipErrorInvalidValue, "push: object box outside the node table");
	unsigned nb = (unsigned)ceil_div(n, kPushChunk);
	*nBlocks = (int)nb;
	hipStream_t st = (hipStream_t)stream;
	const bool kick = args->kick != 0;
	if (kick && !args->Es) return set_error(hipErrorInvalidValue, "push: kick without E");
	// a sorting push never counts (its brick counters use the count's LDS)
	if (sort) a.cntNext = nullptr;
#define LAUNCH_PUSH(ND, V3D, OBJ)                                                                                       \
	do {                                                                                                                \
		if (kick && sort) hipLaunchKernelGGL((k_push<ND, V3D, true, true, OBJ>), dim3(nb), dim3(kPushThreads), 0, st, a); \
		else if (kick) hipLaunchKernelGGL((k_push<ND, V3D, true, false, OBJ>), dim3(nb), dim3(kPushThreads), 0, st, a);   \
		else if (sort) hipLaunchKernelGGL((k_push<ND, V3D, false, true, OBJ>), dim3(nb), dim3(kPushThreads), 0, st, a);   \
		else hipLaunchKernelGGL((k_push<ND, V3D, false, false, OBJ>), dim3(nb), dim3(kPushThreads), 0, st, a);            \
	} while (0)
	if (nd == 3 && a.objIn) LAUNCH_PUSH(3, true, true);
	else if (nd == 3) LAUNCH_PUSH(3, true, false);
	else if (nd == 2) LAUNCH_PUSH(2, false, false);
	else LAUNCH_PUSH(1, false, false);
#undef LAUNCH_PUSH
	return check_launch("push");
}

extern "C" long pinc_hip_tile_keys(pinc_geom_t g, int tileWidth) {
	long nk = 0;
	(void)make_tile_geo(g, tileWidth, &nk);
	return nk;
}

extern "C" int pinc_hip_count_keys(pinc_pop_t pop, int s, long first, pinc_geom_t g, int tileWidth, int *counts,
                                   void *stream) {
	long b0 = pop.iStart[s] + first;
	long n = pop.iStop[s] - b0;
	if (n <= 0) return 0;
	long nk = 0;
	TileGeo tg = make_tile_geo(g, tileWidth, &nk);
	long nb = ceil_div(n, (long)kThreads);
	if (nb > 65536L * 8) nb = 65536L * 8;
	int nd = g.nd;
	const double *x0 = pop.x[0] + b0, *x1 = nd > 1 ? pop.x[1] + b0 : nullptr, *x2 = nd > 2 ? pop.x[2] + b0 : nullptr;
	const double *v0 = pop.v[0] + b0, *v1 = nd > 1 ? pop.v[1] + b0 : nullptr, *v2 = nd > 2 ? pop.v[2] + b0 : nullptr;
	hipStream_t st = (hipStream_t)stream;
	if (nd == 3)
		hipLaunchKernelGGL(k_count_bricks<3>, dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, v0, v1, v2, n, tg, counts);
	else if (nd == 2)
		hipLaunchKernelGGL(k_count_bricks<2>, dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, v0, v1, v2, n, tg, counts);
	else hipLaunchKernelGGL(k_count_bricks<1>, dim3(nb), dim3(kThreads), 0, st, x0, x1, x2, v0, v1, v2, n, tg, counts);
	return check_launch("count_keys");
}

extern "C" int pinc_hip_scan_keys(const int *counts, long nKeys, int *offsets, int *work, void *stream) {
	long nsb = ceil_div(nKeys, (long)kScanBlock);
	if (nsb > 1024L * 1024L) return set_error(hipErrorInvalidValue, "scan_keys: too many keys");
	int *bsum = work, *boff = work + nsb;
	hipStream_t st = (hipStream_t)stream;
	hipLaunchKernelGGL(k_scan_sums, dim3((unsigned)nsb), dim3(kThreads), 0, st, counts, nKeys, bsum);
	hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(1024), 0, st, bsum, boff, (int)nsb);
	hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nsb), dim3(kThreads), 0, st, counts, nKeys, boff, offsets);
	return check_launch("scan_keys");
}


extern "C" int pinc_hip_rho_combine(double *rho, const double *const *acc, const double *charge, int ns, long n,
                                    void *stream) {
	if (ns < 1 || ns > PINC_MAX_SPECIES) return set_error(hipErrorInvalidValue, "rho_combine: species");
	CombineArgs c;
	c.ns = ns;
	for (int s = 0; s < PINC_MAX_SPECIES; s++) {
		c.acc[s] = s < ns ? acc[s] : nullptr;
		c.q[s] = s < ns ? charge[s] : 1.0;
	}
	long nb = ceil_div(n, (long)kThreads * 4);
	if (nb > 8192) nb = 8192;
	hipLaunchKernelGGL(k_rho_combine, dim3((unsigned)nb), dim3(kThreads), 0, (hipStream_t)stream, rho, c, n);
	return check_launch("rho_combine");
}
