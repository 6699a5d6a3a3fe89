// k_mg.hip -- multigrid Poisson kernels for MI355X (gfx950), periodic grid
// without ghost cells (every halo of the reference is an index wrap here).
//
//   gs_pass        one colour of mgGS3D (multigrid.c:683-767) or mgGSND
//                  (553-621).  The reference neutralises phi after every
//                  colour (gBnd -> gNeutralizeGrid, grid.c:730-779).  Here the
//                  mean is subtracted lazily: the colour that was just
//                  written is stored raw with its pending mean mu, and every
//                  read of it evaluates (raw - mu) -- the same rounding as
//                  the reference's stored value.  Each pass also produces the
//                  block partial sums of the resulting grid, from which the
//                  next mean is formed.
//   materialize    applies the pending means after the last pass
//   residual       mgResidual + gFinDiff2nd3D/ND (multigrid.c:1385-1403,
//                  grid.c:264-334)
//   restrict       mgHalfRestrict3D (1/12 weights) / ND (multigrid.c:844-1022)
//   prolong_add    mgBilinProl3D/ND followed by gAddTo (multigrid.c:1024-1238,
//                  1535): the separable z, y, x interpolation is evaluated in
//                  registers with the reference's intermediate roundings.
#include "common.h"

using namespace pinc;

namespace {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 2048;

inline long ceil_div(long a, long b) { return (a + b - 1) / b; }


// 1: the 3-D residual norm on x pairs (k_residual_sumsq3p)
#ifndef PINC_MG_NORM_PAIRS
#define PINC_MG_NORM_PAIRS 1
#endif
// 1: the level-0 residual and restriction on x pairs (k_resid_restrict3p)
#ifndef PINC_MG_RR_PAIRS
#define PINC_MG_RR_PAIRS 1
#endif

struct Lv {
	int T[3];
	long s[3];
};

__device__ __forceinline__ Lv make_lv(const pinc_lvl_t &L) {
	Lv r;
	for (int d = 0; d < 3; d++) r.T[d] = L.T[d];
	r.s[0] = 1;
	r.s[1] = L.T[0];
	r.s[2] = (long)L.T[0] * L.T[1];
	return r;
}

// neighbour offsets of point (c) along dim d with periodic wrap
__device__ __forceinline__ long nb_up(const Lv &L, const int *c, int d) {
	return (c[d] + 1 < L.T[d]) ? L.s[d] : -(long)(L.T[d] - 1) * L.s[d];
}
__device__ __forceinline__ long nb_dn(const Lv &L, const int *c, int d) {
	return (c[d] > 0) ? -L.s[d] : (long)(L.T[d] - 1) * L.s[d];
}

template <int ND, bool GS3D>
__global__ __launch_bounds__(kThreads) void k_gs_pass(double *__restrict__ phi,
                                                      const double *__restrict__ rho, pinc_lvl_t Lp,
                                                      int pass, const double *__restrict__ muPrev,
                                                      double *__restrict__ partial) {
	__shared__ double red[kThreads / 64];
	Lv L = make_lv(Lp);
	double mu = muPrev ? *muPrev : 0.0;
	long half = L.T[0] / 2;
	long nPairs = half * L.T[1] * L.T[2];
	double acc = 0.;
	for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < nPairs; q += (long)gridDim.x * blockDim.x) {
		int c[3];
		const unsigned uq = (unsigned)q, uh = (unsigned)half, t1 = (unsigned)L.T[1];
		const unsigned r = uq / uh;  // 32-bit index arithmetic (levels hold < 2^31 points)
		int i = (int)(uq - r * uh);
		c[1] = (int)(r % t1);
		c[2] = (int)(r / t1);
		int par = (pass + c[1] + c[2]) & 1;
		c[0] = 2 * i + par;            // point of the colour being updated
		int xo = 2 * i + 1 - par;      // point of the other colour
		long g = (long)c[0] + c[1] * L.s[1] + c[2] * L.s[2];
		double v;
		if (GS3D) {
			double xp = phi[g + nb_up(L, c, 0)] - mu, xm = phi[g + nb_dn(L, c, 0)] - mu;
			double yp = phi[g + nb_up(L, c, 1)] - mu, ym = phi[g + nb_dn(L, c, 1)] - mu;
			double zp = phi[g + nb_up(L, c, 2)] - mu, zm = phi[g + nb_dn(L, c, 2)] - mu;
			v = (1. / 6.) * (xp + xm + yp + ym + zp + zm + rho[g]);
		} else {
			v = 0;
#pragma unroll
			for (int d = 0; d < ND; d++) {
				double a = phi[g + nb_up(L, c, d)] - mu, b = phi[g + nb_dn(L, c, d)] - mu;
				v += a + b;
			}
			v += rho[g];
			v *= 1. / (2 * ND);
		}
		phi[g] = v;
		if (partial) {
			long go = g + (xo - c[0]);
			acc += v + (phi[go] - mu);
		}
	}
	// native mode passes no partials: no neutralisation after each colour
	if (!partial) return;
	double t = block_sum(acc, red);
	if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ void k_gs_materialize(double *__restrict__ phi, pinc_lvl_t Lp, int lastPass,
                                 const double *__restrict__ muA, const double *__restrict__ muB) {
	Lv L = make_lv(Lp);
	long n = (long)L.T[0] * L.T[1] * L.T[2];
	double a = muA ? *muA : 0.0, b = *muB;
	for (long g = (long)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (long)gridDim.x * blockDim.x) {
		const unsigned u = (unsigned)g, t0 = (unsigned)L.T[0], t1 = (unsigned)L.T[1];
		const unsigned r = u / t0;
		int x = (int)(u - r * t0);
		int y = (int)(r % t1), z = (int)(r / t1);
		if (((x + y + z) & 1) == lastPass) phi[g] = phi[g] - b;
		else phi[g] = (phi[g] - a) - b;
	}
}

template <int ND>
__device__ __forceinline__ double residual_at(const double *__restrict__ phi,
                                              const double *__restrict__ rho, const Lv &L,
                                              const int *c, long g) {
	double r;
	if (ND == 3) {
		r = -6. * phi[g];
		r += phi[g + nb_up(L, c, 0)] + phi[g + nb_dn(L, c, 0)] + phi[g + nb_up(L, c, 1)] +
		     phi[g + nb_dn(L, c, 1)] + phi[g + nb_up(L, c, 2)] + phi[g + nb_dn(L, c, 2)];
	} else {
		r = -(2. * ND) * phi[g];
#pragma unroll
		for (int d = 0; d < ND; d++) r += phi[g + nb_up(L, c, d)] + phi[g + nb_dn(L, c, d)];
	}
	return r + rho[g];
}

template <int ND>
__global__ void k_residual(double *__restrict__ res, const double *__restrict__ phi,
                           const double *__restrict__ rho, pinc_lvl_t Lp) {
	Lv L = make_lv(Lp);
	long n = (long)L.T[0] * L.T[1] * L.T[2];
	const Walk w = point_walk(n);
	for (long g = w.g0; g < w.g1; g += w.step) {
		int c[3];
		{  // 32-bit index arithmetic (levels hold < 2^31 points, checked on the host)
			const unsigned u = (unsigned)g, t0 = (unsigned)L.T[0], t1 = (unsigned)L.T[1];
			const unsigned r = u / t0;
			c[0] = (int)(u - r * t0);
			c[1] = (int)(r % t1);
			c[2] = (int)(r / t1);
		}
		res[g] = residual_at<ND>(phi, rho, L, c, g);
	}
}

template <int ND>
__global__ __launch_bounds__(kThreads) void k_residual_sumsq(const double *__restrict__ phi,
                                                             const double *__restrict__ rho,
                                                             pinc_lvl_t Lp,
                                                             double *__restrict__ partial) {
	__shared__ double red[kThreads / 64];
	Lv L = make_lv(Lp);
	long n = (long)L.T[0] * L.T[1] * L.T[2];
	double acc = 0.;
	const Walk w = point_walk(n);
	for (long g = w.g0; g < w.g1; g += w.step) {
		int c[3];
		{  // 32-bit index arithmetic (levels hold < 2^31 points, checked on the host)
			const unsigned u = (unsigned)g, t0 = (unsigned)L.T[0], t1 = (unsigned)L.T[1];
			const unsigned r = u / t0;
			c[0] = (int)(u - r * t0);
			c[1] = (int)(r % t1);
			c[2] = (int)(r / t1);
		}
		double v = residual_at<ND>(phi, rho, L, c, g);
		acc += v * v;
	}
	double t = block_sum(acc, red);
	if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

// k_residual_sumsq<3> on x pairs (x even): the point and its x+1 neighbour,
// and the pairs of the y and z neighbour rows, as 16-B loads, the outer x
// neighbours as 8-B loads.  Each residual is residual_at's expression in its
// order; only the order of the squares' sum differs.  Levels with an even x
// extent and 16-B aligned arrays.
__global__ __launch_bounds__(kThreads) void k_residual_sumsq3p(const double *__restrict__ phi,
                                                               const double *__restrict__ rho, pinc_lvl_t Lp,
                                                               double *__restrict__ partial) {
	__shared__ double red[kThreads / 64];
	const unsigned T0 = Lp.T[0], T1 = Lp.T[1], T2 = Lp.T[2];
	const unsigned hx = T0 / 2;
	const long sy = T0, sz = (long)T0 * T1;
	const long n2 = (long)hx * T1 * T2;
	double acc = 0.;
	const Walk w = point_walk(n2);
	for (long q = w.g0; q < w.g1; q += w.step) {
		const unsigned u = (unsigned)q, r = u / hx;
		const int x = 2 * (int)(u - r * hx), y = (int)(r % T1), z = (int)(r / T1);
		const long g = (long)x + y * sy + z * sz;
		const long oym = y > 0 ? -sy : (long)(T1 - 1) * sy, oyp = y + 1 < (int)T1 ? sy : -(long)(T1 - 1) * sy;
		const long ozm = z > 0 ? -sz : (long)(T2 - 1) * sz, ozp = z + 1 < (int)T2 ? sz : -(long)(T2 - 1) * sz;
		const long oxm = x > 0 ? -1 : (long)T0 - 1, oxp = x + 2 < (int)T0 ? 2 : 2 - (long)T0;
		const double2 c = *reinterpret_cast<const double2 *>(phi + g);
		const double2 pr = *reinterpret_cast<const double2 *>(rho + g);
		const double2 ym = *reinterpret_cast<const double2 *>(phi + g + oym);
		const double2 yp = *reinterpret_cast<const double2 *>(phi + g + oyp);
		const double2 zm = *reinterpret_cast<const double2 *>(phi + g + ozm);
		const double2 zp = *reinterpret_cast<const double2 *>(phi + g + ozp);
		const double xm0 = phi[g + oxm], xp1 = phi[g + oxp];
		// residual_at<3>: -6 phi + (x+ + x- + y+ + y- + z+ + z-) + rho
		double r0 = -6. * c.x;
		r0 += c.y + xm0 + yp.x + ym.x + zp.x + zm.x;
		r0 = r0 + pr.x;
		double r1 = -6. * c.y;
		r1 += xp1 + c.x + yp.y + ym.y + zp.y + zm.y;
		r1 = r1 + pr.y;
		acc += r0 * r0;
		acc += r1 * r1;
	}
	double t = block_sum(acc, red);
	if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

template <int ND, bool HW3D>
__global__ void k_restrict(const double *__restrict__ fine, double *__restrict__ coarse, pinc_lvl_t Lc) {
	Lv C = make_lv(Lc);
	pinc_lvl_t Lfp = Lc;
	for (int d = 0; d < ND; d++) Lfp.T[d] = 2 * Lc.T[d];
	Lv F = make_lv(Lfp);
	long n = (long)C.T[0] * C.T[1] * C.T[2];
	const Walk w = point_walk(n);
	for (long gc = w.g0; gc < w.g1; gc += w.step) {
		int cc[3], cf[3] = {0, 0, 0};
		{  // 32-bit index arithmetic (levels hold < 2^31 points, checked on the host)
			const unsigned u = (unsigned)gc, t0 = (unsigned)C.T[0], t1 = (unsigned)C.T[1];
			const unsigned r = u / t0;
			cc[0] = (int)(u - r * t0);
			cc[1] = (int)(r % t1);
			cc[2] = (int)(r / t1);
		}
		long gf = 0;
		for (int d = 0; d < ND; d++) {
			cf[d] = 2 * cc[d];
			gf += (long)cf[d] * F.s[d];
		}
		double v;
		if (HW3D) {
			v = (1. / 12.) * (6 * fine[gf] + fine[gf + nb_up(F, cf, 0)] + fine[gf + nb_dn(F, cf, 0)] +
			                  fine[gf + nb_up(F, cf, 1)] + fine[gf + nb_dn(F, cf, 1)] +
			                  fine[gf + nb_up(F, cf, 2)] + fine[gf + nb_dn(F, cf, 2)]);
		} else {
			v = (2. * ND) * fine[gf];
#pragma unroll
			for (int d = 0; d < ND; d++) v += fine[gf + nb_up(F, cf, d)] + fine[gf + nb_dn(F, cf, d)];
			v *= 1. / (ND * 4);
		}
		coarse[gc] = v;
	}
}

// Value of the prolongated coarse grid at fine point cf.  The reference
// interpolates the highest dimension first (z, then y, then x, each pass
// preceded by a TOHALO of that dimension), so a point that is odd in several
// dimensions is the average, along its LOWEST odd dimension, of values
// already interpolated along the higher ones.  Evaluating from dim 0 upward
// reproduces every intermediate rounding of the reference.
template <int ND, int D>
__device__ __forceinline__ double prol_low(const double *__restrict__ cv, const Lv &C, const int *cf) {
	if constexpr (D == ND) {
		long g = 0;
		for (int d = 0; d < ND; d++) g += (long)(cf[d] >> 1) * C.s[d];
		return cv[g];
	} else {
		if (!(cf[D] & 1)) return prol_low<ND, D + 1>(cv, C, cf);
		int a[3] = {cf[0], cf[1], cf[2]}, b[3] = {cf[0], cf[1], cf[2]};
		a[D] = cf[D] - 1;
		b[D] = cf[D] + 1;
		if (b[D] >= 2 * C.T[D]) b[D] -= 2 * C.T[D];
		return 0.5 * (prol_low<ND, D + 1>(cv, C, a) + prol_low<ND, D + 1>(cv, C, b));
	}
}

template <int ND>
__global__ void k_prolong_add(double *__restrict__ phiF, const double *__restrict__ phiC, pinc_lvl_t Lf) {
	pinc_lvl_t Lcp = Lf;
	for (int d = 0; d < ND; d++) Lcp.T[d] = Lf.T[d] / 2;
	Lv C = make_lv(Lcp);
	Lv F = make_lv(Lf);
	long n = (long)F.T[0] * F.T[1] * F.T[2];
	const Walk w = point_walk(n);
	for (long g = w.g0; g < w.g1; g += w.step) {
		int cf[3];
		{  // 32-bit index arithmetic (levels hold < 2^31 points, checked on the host)
			const unsigned u = (unsigned)g, t0 = (unsigned)F.T[0], t1 = (unsigned)F.T[1];
			const unsigned r = u / t0;
			cf[0] = (int)(u - r * t0);
			cf[1] = (int)(r % t1);
			cf[2] = (int)(r / t1);
		}
		phiF[g] += prol_low<ND, 0>(phiC, C, cf);
	}
}

inline unsigned blocks_for(long n) {
	long b = ceil_div(n, (long)kThreads * 4);
	if (b < 1) b = 1;
	if (b > kMaxBlocks) b = kMaxBlocks;
	return (unsigned)b;
}

inline long npts(const pinc_lvl_t &L) { return (long)L.T[0] * L.T[1] * L.T[2]; }


// ------------------------------------------------ fused red-black sweep ---
// One full red-black Gauss-Seidel iteration of mgGS3D (red = storage
// (x+y+z) even first, then black; the 1/6 * left-to-right sum of the six
// neighbours and rho) in a single pass, from phiIn to phiOut, without the
// per-colour neutralisation (native mode only; multigrid:native).  Each
// workgroup owns a 16x16 column tile and a chunk of kSwZ planes, marching
// in z with a 4-plane LDS ring: red of plane z+1 (on the tile plus a one-node
// halo, recomputed redundantly, from old black values) is formed before
// black of plane z (from new red).  Every value read from memory is an old
// one, so the result equals the two-pass iteration bit for bit, and each
// sweep reads phi and rho and writes phi once (24 B per point) instead of
// twice per colour.
constexpr int kSwT = 16;       // tile side (x, y)
constexpr int kSwH = kSwT + 4; // with the two-node halo
constexpr int kSwR = kSwT + 2; // red region: tile plus one
constexpr int kSwZ = 16;       // planes per workgroup


// XCD-aware tile order for the z-marching sweeps (PINC_MG_XCD): blocks are
// dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup
// dispatch), so block b runs on XCD b % 8.  Map it to tile
// x*q + min(x, r) + y (x = b % 8, y = b / 8) so that each XCD sweeps a
// contiguous run of tiles, whose x and y halo reads are its neighbours'
// interiors in the same L2.  A bijection for any grid, placement only.
// Measured neutral at C4 (k_gs_sweep4 0.192 ms either way: the march is
// latency-bound, not L2-miss bound), so off by default.
#ifndef PINC_MG_S4_SPLIT
#define PINC_MG_S4_SPLIT 1
#endif
#ifndef PINC_MG_SWEEP4C
#define PINC_MG_SWEEP4C 1
#endif
#ifndef PINC_MG_XCD
#define PINC_MG_XCD 0
#endif
__device__ __forceinline__ unsigned xcd_tile(unsigned b, unsigned nb) {
#if PINC_MG_XCD
	const unsigned x = b & 7u, y = b >> 3, q = nb >> 3, r = nb & 7u;
	return x * q + min(x, r) + y;
#else
	(void)nb;
	return b;
#endif
}

__global__ __launch_bounds__(256) void k_gs_sweep(const double *__restrict__ phiIn,
                                                  double *__restrict__ phiOut,
                                                  const double *__restrict__ rho, pinc_lvl_t Lp) {
	// 5-plane phi ring and 3-plane rho ring: the next planes are prefetched
	// into registers while the current ones are relaxed, two barriers per plane
	__shared__ double cur[5][kSwH][kSwH];
	__shared__ double rh[3][kSwR][kSwR];
	const int TX = Lp.T[0], TY = Lp.T[1], TZ = Lp.T[2];
	const long sy = TX, sz = (long)TX * TY;
	const int ntx = TX / kSwT, nty = TY / kSwT;
	const unsigned tb = xcd_tile(blockIdx.x, gridDim.x);
	const int bx = tb % ntx, by = (tb / ntx) % nty, bz = tb / (ntx * nty);
	const int x0 = bx * kSwT, y0 = by * kSwT, z0 = bz * kSwZ;
	const int tid = threadIdx.x;
	auto wrapi = [](int i, int T) { return i < 0 ? i + T : (i >= T ? i - T : i); };
	auto gidx = [&](int x, int y, int z) {
		return (long)wrapi(x, TX) + wrapi(y, TY) * sy + (long)wrapi(z, TZ) * sz;
	};
	auto ps = [](int z) { return (z + 10) % 5; };
	auto rs = [](int z) { return (z + 9) % 3; };
	// this thread's share of a plane: phi items tid, tid+256 (< 400), rho
	// items tid, tid+256 (< 324)
	auto fetch_phi = [&](int z, double *f) {
		for (int k = 0; k < 2; k++) {
			int i = tid + 256 * k;
			if (i < kSwH * kSwH) f[k] = phiIn[gidx(x0 + i % kSwH - 2, y0 + i / kSwH - 2, z)];
		}
	};
	auto fetch_rho = [&](int z, double *r) {
		for (int k = 0; k < 2; k++) {
			int i = tid + 256 * k;
			if (i < kSwR * kSwR) r[k] = rho[gidx(x0 + i % kSwR - 1, y0 + i / kSwR - 1, z)];
		}
	};
	auto put = [&](int zf, int zr, const double *f, const double *r, bool withRho) {
		for (int k = 0; k < 2; k++) {
			int i = tid + 256 * k;
			if (i < kSwH * kSwH) cur[ps(zf)][i / kSwH][i % kSwH] = f[k];
			if (withRho && i < kSwR * kSwR) rh[rs(zr)][i / kSwR][i % kSwR] = r[k];
		}
	};
	// red points of plane z on the tile (+ one-node halo if wide)
	auto red = [&](int z, bool wide) {
		double(*c)[kSwH] = cur[ps(z)];
		double(*cm)[kSwH] = cur[ps(z - 1)];
		double(*cp)[kSwH] = cur[ps(z + 1)];
		double(*r)[kSwR] = rh[rs(z)];
		const int lo = wide ? 0 : 1, w = wide ? kSwR : kSwT;
		for (int i = tid; i < w * w; i += 256) {
			int hx = lo + i % w, hy = lo + i / w;  // red-region coordinates
			int gx = x0 + hx - 1, gy = y0 + hy - 1;
			if (((gx + gy + z) & 1) != 0) continue;
			int cx = hx + 1, cy = hy + 1;          // ring coordinates
			double xp = c[cy][cx + 1], xm = c[cy][cx - 1];
			double yp = c[cy + 1][cx], ym = c[cy - 1][cx];
			double zp = cp[cy][cx], zm = cm[cy][cx];
			c[cy][cx] = (1. / 6.) * (xp + xm + yp + ym + zp + zm + r[hy][hx]);
		}
	};

	// prologue: planes z0-2 .. z0+2 and rho z0-1 .. z0+1 in LDS, red of
	// z0-1 (tile) and z0 (wide)
	{
		double f[2], r[2];
		for (int z = z0 - 2; z <= z0 + 2; z++) {
			fetch_phi(z, f);
			if (z >= z0 - 1 && z <= z0 + 1) fetch_rho(z, r);
			put(z, z, f, r, z >= z0 - 1 && z <= z0 + 1);
		}
	}
	__syncthreads();
	red(z0 - 1, false);
	__syncthreads();
	red(z0, true);
	__syncthreads();
	const int tx = tid % kSwT, ty = tid / kSwT;
	for (int z = z0; z < z0 + kSwZ; z++) {
		// LDS: phi planes z-2 .. z+2, rho planes z-1 .. z+1
		double f[2], r[2];
		fetch_phi(z + 3, f);  // in flight during the relaxation below
		fetch_rho(z + 2, r);
		red(z + 1, true);
		__syncthreads();
		double(*c)[kSwH] = cur[ps(z)];
		double(*cm)[kSwH] = cur[ps(z - 1)];
		double(*cp)[kSwH] = cur[ps(z + 1)];
		int gx = x0 + tx, gy = y0 + ty;
		int cx = tx + 2, cy = ty + 2;
		double v = c[cy][cx];
		if (((gx + gy + z) & 1) != 0) {
			double xp = c[cy][cx + 1], xm = c[cy][cx - 1];
			double yp = c[cy + 1][cx], ym = c[cy - 1][cx];
			double zp = cp[cy][cx], zm = cm[cy][cx];
			v = (1. / 6.) * (xp + xm + yp + ym + zp + zm + rh[rs(z)][ty + 1][tx + 1]);
		}
		phiOut[gidx(gx, gy, z)] = v;
		// slot of phi z+3 held z-2 (last read by black z-1), slot of rho z+2
		// held z-1 (last read by red z-1): both free since the barrier above
		put(z + 3, z + 2, f, r, true);
		__syncthreads();
	}
}


// Variant of k_gs_sweep with the planes fetched two iterations ahead of
// their use (the HBM latency of a plane is covered by two plane
// relaxations), tile SX x SY per NT-thread workgroup.  Same ring scheme and
// the same arithmetic as k_gs_sweep (bit-identical results).
template <int SX, int SY, int NT>
struct Sweep2 {
	static constexpr int HX = SX + 4, HY = SY + 4;  // phi region (two-node halo)
	static constexpr int RX = SX + 2, RY = SY + 2;  // red region (one-node halo)
	static constexpr int PhiSlots = (HX * HY + NT - 1) / NT;
	static constexpr int RhoSlots = (RX * RY + NT - 1) / NT;
};

template <int kS2X, int kS2Y, int kS2Threads>
__global__ __launch_bounds__(kS2Threads) void k_gs_sweep2(const double *__restrict__ phiIn,
                                                          double *__restrict__ phiOut,
                                                          const double *__restrict__ rho, pinc_lvl_t Lp,
                                                          int zPlanes) {
	using S = Sweep2<kS2X, kS2Y, kS2Threads>;
	constexpr int kS2HX = S::HX, kS2HY = S::HY, kS2RX = S::RX, kS2RY = S::RY;
	constexpr int kS2PhiSlots = S::PhiSlots, kS2RhoSlots = S::RhoSlots;
	__shared__ double cur[5][kS2HY][kS2HX];
	__shared__ double rh[3][kS2RY][kS2RX];
	const int TX = Lp.T[0], TY = Lp.T[1], TZ = Lp.T[2];
	const long sy = TX, sz = (long)TX * TY;
	const int ntx = TX / kS2X, nty = TY / kS2Y;
	const unsigned tb = xcd_tile(blockIdx.x, gridDim.x);
	const int bx = tb % ntx, by = (tb / ntx) % nty, bz = tb / (ntx * nty);
	const int x0 = bx * kS2X, y0 = by * kS2Y, z0 = bz * zPlanes;
	const int tid = threadIdx.x;
	auto wrapi = [](int i, int T) { return i < 0 ? i + T : (i >= T ? i - T : i); };
	auto gidx = [&](int x, int y, int z) {
		return (long)wrapi(x, TX) + wrapi(y, TY) * sy + (long)wrapi(z, TZ) * sz;
	};
	auto ps = [](int z) { return (z + 10) % 5; };
	auto rs = [](int z) { return (z + 9) % 3; };
	auto fetch = [&](int zf, int zr, double *f, double *r) {
#pragma unroll
		for (int k = 0; k < kS2PhiSlots; k++) {
			int i = tid + kS2Threads * k;
			if (i < kS2HX * kS2HY) f[k] = phiIn[gidx(x0 + i % kS2HX - 2, y0 + i / kS2HX - 2, zf)];
		}
#pragma unroll
		for (int k = 0; k < kS2RhoSlots; k++) {
			int i = tid + kS2Threads * k;
			if (i < kS2RX * kS2RY) r[k] = rho[gidx(x0 + i % kS2RX - 1, y0 + i / kS2RX - 1, zr)];
		}
	};
	auto put = [&](int zf, int zr, const double *f, const double *r) {
#pragma unroll
		for (int k = 0; k < kS2PhiSlots; k++) {
			int i = tid + kS2Threads * k;
			if (i < kS2HX * kS2HY) cur[ps(zf)][i / kS2HX][i % kS2HX] = f[k];
		}
#pragma unroll
		for (int k = 0; k < kS2RhoSlots; k++) {
			int i = tid + kS2Threads * k;
			if (i < kS2RX * kS2RY) rh[rs(zr)][i / kS2RX][i % kS2RX] = r[k];
		}
	};
	auto red = [&](int z, bool wide) {
		double(*c)[kS2HX] = cur[ps(z)];
		double(*cm)[kS2HX] = cur[ps(z - 1)];
		double(*cp)[kS2HX] = cur[ps(z + 1)];
		double(*r)[kS2RX] = rh[rs(z)];
		const int lo = wide ? 0 : 1, wx = wide ? kS2RX : kS2X, wy = wide ? kS2RY : kS2Y;
		for (int i = tid; i < wx * wy; i += kS2Threads) {
			int hx = lo + i % wx, hy = lo + i / wx;  // red-region coordinates
			int gx = x0 + hx - 1, gy = y0 + hy - 1;
			if (((gx + gy + z) & 1) != 0) continue;
			int cx = hx + 1, cy = hy + 1;          // ring coordinates
			double xp = c[cy][cx + 1], xm = c[cy][cx - 1];
			double yp = c[cy + 1][cx], ym = c[cy - 1][cx];
			double zp = cp[cy][cx], zm = cm[cy][cx];
			c[cy][cx] = (1. / 6.) * (xp + xm + yp + ym + zp + zm + r[hy][hx]);
		}
	};

	// prologue: phi z0-2 .. z0+2 and rho z0-1 .. z0+1 into LDS, phi z0+3 and
	// rho z0+2 into registers (set A); red of z0-1 (tile) and z0 (wide)
	double fa[kS2PhiSlots], ra[kS2RhoSlots], fb[kS2PhiSlots], rb[kS2RhoSlots];
	for (int z = z0 - 2; z <= z0 + 2; z++) {
		fetch(z, z, fb, rb);
		if (z >= z0 - 1 && z <= z0 + 1) put(z, z, fb, rb);
		else {
#pragma unroll
			for (int k = 0; k < kS2PhiSlots; k++) {
				int i = tid + kS2Threads * k;
				if (i < kS2HX * kS2HY) cur[ps(z)][i / kS2HX][i % kS2HX] = fb[k];
			}
		}
	}
	fetch(z0 + 3, z0 + 2, fa, ra);
	__syncthreads();
	red(z0 - 1, false);
	__syncthreads();
	red(z0, true);
	__syncthreads();
	const int tx = tid % kS2X, ty = tid / kS2X;
	for (int z = z0; z < z0 + zPlanes; z++) {
		// LDS: phi z-2 .. z+2, rho z-1 .. z+1; registers A: phi z+3, rho z+2
		fetch(z + 4, z + 3, fb, rb);  // two iterations ahead of its use
		red(z + 1, true);
		__syncthreads();
		double(*c)[kS2HX] = cur[ps(z)];
		double(*cm)[kS2HX] = cur[ps(z - 1)];
		double(*cp)[kS2HX] = cur[ps(z + 1)];
		int gx = x0 + tx, gy = y0 + ty;
		int cx = tx + 2, cy = ty + 2;
		double v = c[cy][cx];
		if (((gx + gy + z) & 1) != 0) {
			double xp = c[cy][cx + 1], xm = c[cy][cx - 1];
			double yp = c[cy + 1][cx], ym = c[cy - 1][cx];
			double zp = cp[cy][cx], zm = cm[cy][cx];
			v = (1. / 6.) * (xp + xm + yp + ym + zp + zm + rh[rs(z)][ty + 1][tx + 1]);
		}
		phiOut[gidx(gx, gy, z)] = v;
		// phi z+3 into the slot of z-2 (last read by black z-1), rho z+2 into
		// the slot of z-1 (last read by red z-1)
		put(z + 3, z + 2, fa, ra);
		__syncthreads();
#pragma unroll
		for (int k = 0; k < kS2PhiSlots; k++) fa[k] = fb[k];
#pragma unroll
		for (int k = 0; k < kS2RhoSlots; k++) ra[k] = rb[k];
	}
}

// ------------------------------------ two red-black iterations per launch ---
// The same z-march as k_gs_sweep2, four stages deep.  At step s the
// workgroup updates, in a first phase, red (1st iteration) on plane s+3, red
// (2nd) on s and black (2nd) on s-2, which it writes out; then, after one
// barrier, black (1st) on s+2.  The stages of a phase only read planes the
// others do not write, and each reads the phi plane ring as the stage before
// it left it (in place: a stage overwrites only values no later stage
// needs), so a step costs two barriers.  Each stage is computed on a region
// one node wider than the next, so the tile needs a four-node halo and no
// exchange with its neighbours.  rho is not staged: every thread loads the
// rho values of its own stage nodes two steps ahead into registers, which
// keeps the LDS at 40 KB and four workgroups on a CU (the march is
// latency-bound: a step waits for loads issued two steps earlier).  phiIn is read and phiOut
// written once per two iterations; the arithmetic is that of mgGS3D's red
// and black passes, so the result is bit-identical to two k_gs_sweep2
// launches.
template <int SX, int SY, int NT>
struct Sweep4 {
	static constexpr int H = 4;  // phi halo
	static constexpr int HX = SX + 2 * H, HY = SY + 2 * H;
	static constexpr int NP = 8;  // ring planes
	static constexpr int PhiSlots = (HX * HY + NT - 1) / NT;
	// nodes of one colour on the tile grown by h (rows have even length)
	static constexpr int nodes(int h) { return (SX + 2 * h) / 2 * (SY + 2 * h); }
	static constexpr int K3 = (nodes(3) + NT - 1) / NT, K2 = (nodes(2) + NT - 1) / NT,
	                     K1 = (nodes(1) + NT - 1) / NT;
};

template <int SX, int SY, int NT>
__global__ __launch_bounds__(NT) void k_gs_sweep4(const double *__restrict__ phiIn, double *__restrict__ phiOut,
                                                  const double *__restrict__ rho, pinc_lvl_t Lp, int zPlanes) {
	using S = Sweep4<SX, SY, NT>;
	constexpr int HX = S::HX, HY = S::HY, H = S::H, K3 = S::K3, K2 = S::K2, K1 = S::K1;
	__shared__ double cur[S::NP][HY][HX];
	const int TX = Lp.T[0], TY = Lp.T[1], TZ = Lp.T[2];
	const long sy = TX, sz = (long)TX * TY;
	const int ntx = TX / SX, nty = TY / SY;
	const unsigned tb = xcd_tile(blockIdx.x, gridDim.x);
	const int bx = tb % ntx, by = (tb / ntx) % nty, bz = tb / (ntx * nty);
	const int x0 = bx * SX, y0 = by * SY, z0 = bz * zPlanes;
	const int tid = threadIdx.x;
	auto wrapi = [](int i, int T) { return i < 0 ? i + T : (i >= T ? i - T : i); };
	auto gidx = [&](int x, int y, int z) {
		return (long)wrapi(x, TX) + wrapi(y, TY) * sy + (long)wrapi(z, TZ) * sz;
	};
	auto ps = [](int z) { return (z + 8 * 16) % S::NP; };
	auto fetch = [&](int zf, double *f) {
#pragma unroll
		for (int k = 0; k < S::PhiSlots; k++) {
			int i = tid + NT * k;
			if (i < HX * HY) f[k] = phiIn[gidx(x0 + i % HX - H, y0 + i / HX - H, zf)];
		}
	};
	auto putPhi = [&](int zf, const double *f) {
#pragma unroll
		for (int k = 0; k < S::PhiSlots; k++) {
			int i = tid + NT * k;
			if (i < HX * HY) cur[ps(zf)][i / HX][i % HX] = f[k];
		}
	};
	// node j of colour `parity` on plane p, tile grown by h: tile coordinates
	auto node = [&](int j, int p, int parity, int h, int &tx, int &ty) {
		const int hw = (SX + 2 * h) / 2;
		ty = j / hw - h;
		tx = -h + 2 * (j % hw) + ((parity - (x0 - h + y0 + ty + p)) & 1);
	};
	// rho of this thread's nodes in the four stages of step s
	struct Rho {
		double r1[K3], b1[K2], r2[K1], b2;
	};
	auto fetchRho = [&](int s, Rho &R) {
		int tx, ty;
#pragma unroll
		for (int k = 0; k < K3; k++) {
			const int j = tid + NT * k;
			if (j < S::nodes(3)) {
				node(j, s + 3, 0, 3, tx, ty);
				R.r1[k] = rho[gidx(x0 + tx, y0 + ty, s + 3)];
			}
		}
#pragma unroll
		for (int k = 0; k < K2; k++) {
			const int j = tid + NT * k;
			if (j < S::nodes(2)) {
				node(j, s + 2, 1, 2, tx, ty);
				R.b1[k] = rho[gidx(x0 + tx, y0 + ty, s + 2)];
			}
		}
#pragma unroll
		for (int k = 0; k < K1; k++) {
			const int j = tid + NT * k;
			if (j < S::nodes(1)) {
				node(j, s, 0, 1, tx, ty);
				R.r2[k] = rho[gidx(x0 + tx, y0 + ty, s)];
			}
		}
		R.b2 = rho[gidx(x0 + tid % SX, y0 + tid / SX, s - 2)];
	};
	// colour `parity` of plane p on the tile grown by h, in place
	auto stage = [&](int p, int parity, int h, const double *rv, int nk) {
		double(*c)[HX] = cur[ps(p)];
		double(*cm)[HX] = cur[ps(p - 1)];
		double(*cp)[HX] = cur[ps(p + 1)];
#pragma unroll
		for (int k = 0; k < 2; k++) {
			const int j = tid + NT * k;
			if (k >= nk || j >= S::nodes(h)) break;
			int tx, ty;
			node(j, p, parity, h, tx, ty);
			const int cx = tx + H, cy = ty + H;
			double xp = c[cy][cx + 1], xm = c[cy][cx - 1];
			double yp = c[cy + 1][cx], ym = c[cy - 1][cx];
			double zp = cp[cy][cx], zm = cm[cy][cx];
			c[cy][cx] = (1. / 6.) * (xp + xm + yp + ym + zp + zm + rv[k]);
		}
	};
	static_assert(K3 <= 2 && K2 <= 2 && K1 <= 2, "stage loops are unrolled twice");
	static_assert(SX * SY == NT, "one output node per thread and plane");

	// prologue: phi z0-4 .. z0-2 into LDS, z0-1 into registers A; rho of
	// the first two steps
	double fa[S::PhiSlots], fb[S::PhiSlots];
	for (int z = z0 - 4; z <= z0 - 2; z++) {
		fetch(z, fb);
		putPhi(z, fb);
	}
	fetch(z0 - 1, fa);
	Rho RA, RB, RC;
	fetchRho(z0 - 6, RA);
	fetchRho(z0 - 5, RB);
	__syncthreads();
	const int tx = tid % SX, ty = tid / SX;
	const int zEnd = z0 + zPlanes;  // outputs z0 .. zEnd-1
	for (int s = z0 - 6; s <= zEnd + 1; s++) {
		// LDS: phi s-3 .. s+4 (those each stage reads)
		if (s <= zEnd) {  // two steps ahead of their use
			fetch(s + 6, fb);
			fetchRho(s + 2, RC);
		}
		if (s + 3 <= zEnd + 2) stage(s + 3, 0, 3, RA.r1, K3);          // red, 1st iteration
		if (s >= z0 - 1 && s <= zEnd) stage(s, 0, 1, RA.r2, K1);       // red, 2nd
		if (s - 2 >= z0 && s - 2 < zEnd) {                              // black, 2nd: out
			const int zo = s - 2;
			double(*c)[HX] = cur[ps(zo)];
			double(*cm)[HX] = cur[ps(zo - 1)];
			double(*cp)[HX] = cur[ps(zo + 1)];
			const int gx = x0 + tx, gy = y0 + ty, cx = tx + H, cy = ty + H;
			double v = c[cy][cx];
			if (((gx + gy + zo) & 1) != 0) {
				double xp = c[cy][cx + 1], xm = c[cy][cx - 1];
				double yp = c[cy + 1][cx], ym = c[cy - 1][cx];
				double zp = cp[cy][cx], zm = cm[cy][cx];
				v = (1. / 6.) * (xp + xm + yp + ym + zp + zm + RA.b2);
			}
			phiOut[gidx(gx, gy, zo)] = v;
		}
		__syncthreads();
		if (s + 2 >= z0 - 2 && s + 2 <= zEnd + 1) stage(s + 2, 1, 2, RA.b1, K2);  // black, 1st
		// phi s+5 into the slot of s-3 (last read by the black output above)
		putPhi(s + 5, fa);
		__syncthreads();
#pragma unroll
		for (int k = 0; k < S::PhiSlots; k++) fa[k] = fb[k];
		RA = RB;
		RB = RC;
	}
}

// k_gs_sweep4 restructured for instruction count (same stages, ring and
// arithmetic, bit-identical results).  The profile of k_gs_sweep4 at 256^3
// (profiles/r02s_mg_pmc*.json) is issue-bound, not HBM-bound: per wave 8.7 k
// VALU and 17 k SALU instructions for 72 plane steps, and LDS bank
// conflicts on the checkerboard (lanes two doubles apart).  Here
//   * the LDS ring stores each row split by x parity ([y][x & 1][x >> 1]),
//     so a stage's nodes -- one colour, hence one x parity per row -- and
//     their y and z neighbours are consecutive doubles across lanes, and
//     the two x neighbours are a consecutive pair (one ds_read2);
//   * every per-node LDS index and global rho offset is computed once per
//     thread and plane parity, before the march;
//   * the march is unrolled over the 8 ring planes, so plane slots, plane
//     parities and the phi double buffer are compile-time, and LDS
//     addresses are a per-thread base plus an immediate offset;
//   * global loads are a per-plane scalar base plus a 32-bit byte offset.
template <int SX, int SY, int NT>
struct Sweep4c {
	static constexpr int H = 4;
	static constexpr int HX = SX + 2 * H, HY = SY + 2 * H, HW = HX / 2;
	static constexpr int PL = HX * HY;  // doubles per ring plane
	static constexpr int PhiSlots = (PL + NT - 1) / NT;
	static constexpr int nodes(int h) { return (SX + 2 * h) / 2 * (SY + 2 * h); }
	static_assert(nodes(3) <= 2 * NT && nodes(2) <= NT && nodes(1) <= NT, "stage slots");
	static_assert(SX * SY == NT, "one output node per thread and plane");
	static_assert(PhiSlots == 3, "phi fetch slots");
};

struct S4Node {
	unsigned li, lxm;  // LDS indices of the node and of its x-1 neighbour (x+1 follows)
	unsigned roff;     // byte offset of the node in a plane of the level
};

// diagnostics only (timing by elimination, wrong results): bit 0 skips the
// rho loads, bit 1 the phi fetch, bit 2 pads LDS to two workgroups per CU
#ifndef PINC_MG_S4_DIAG
#define PINC_MG_S4_DIAG 0
#endif
// 1: rho rides in an LDS ring of its own, fetched like phi (three
// row-contiguous loads per thread and step) and read by each stage from its
// node's LDS index; 0: each thread gathers the rho of its four stages' nodes
// from memory (five colour-strided 8-B gathers per step, every value loaded
// four times).  Elimination builds (PINC_MG_S4_DIAG) put the gathers at half
// the launch: 0.168 ms with them, 0.089 ms without, while halving the
// workgroups per CU costs 5 %; the ring takes 80 KB, two workgroups per CU
#ifndef PINC_MG_S4_RHOLDS
#define PINC_MG_S4_RHOLDS 1
#endif
// with the rho ring: phi and rho planes fetched this many steps ahead of
// the step that stores them to LDS minus one (2: plane s+6 at step s; 3:
// s+7, one register set more, for two workgroups per CU)
#ifndef PINC_MG_S4_AHEAD
#define PINC_MG_S4_AHEAD 2
#endif
// 1: the phi and rho plane fetches as 16-B x pairs (two loads per thread
// and plane, the second on the last wave) instead of three 8-B loads
#ifndef PINC_MG_S4_PAIRS
#define PINC_MG_S4_PAIRS 1
#endif
typedef double s4pair __attribute__((ext_vector_type(2)));
template <int SX, int SY, int NT>
__global__ __launch_bounds__(NT) void k_gs_sweep4c(const double *__restrict__ phiIn, double *__restrict__ phiOut,
                                                   const double *__restrict__ rho, pinc_lvl_t Lp, int zPlanes) {
	using S = Sweep4c<SX, SY, NT>;
	constexpr int H = S::H, HX = S::HX, HW = S::HW, PL = S::PL;
	__shared__ double L[8 * PL];
#if PINC_MG_S4_RHOLDS
	__shared__ double Rl[8 * PL];
#endif
#if PINC_MG_S4_DIAG & 4
	__shared__ double padL[38 * 128];
	if (zPlanes < 0) padL[threadIdx.x] = 1.0, phiOut[threadIdx.x] = padL[(threadIdx.x * 7) % (38 * 128)];
#endif
	const int TX = Lp.T[0], TY = Lp.T[1], TZ = Lp.T[2];
	const long sz = (long)TX * TY;
	const int ntx = TX / SX, nty = TY / SY;
	const unsigned tb = xcd_tile(blockIdx.x, gridDim.x);
	const int bx = tb % ntx, by = (tb / ntx) % nty, bz = tb / (ntx * nty);
	const int x0 = bx * SX, y0 = by * SY, z0 = bz * zPlanes;
	const int tid = threadIdx.x;
	auto wrapi = [](int i, int T) { return i < 0 ? i + T : (i >= T ? i - T : i); };
	auto lidx = [](int lx, int ly) { return (unsigned)(ly * HX + (lx & 1) * HW + (lx >> 1)); };
	auto poff = [&](int gx, int gy) { return (unsigned)(wrapi(gx, TX) + wrapi(gy, TY) * TX) * 8u; };
	// node j of colour c on a plane of parity P, tile grown by h (the
	// k_gs_sweep4 enumeration)
	auto mknode = [&](int j, int c, int h, int P) {
		const int hw = (SX + 2 * h) / 2;
		if (j >= S::nodes(h)) j = 0;  // idle lane: any valid node
		const int ty = j / hw - h;
		const int tx = -h + 2 * (j % hw) + ((c - (x0 - h + y0 + ty + P)) & 1);
		S4Node n;
		n.li = lidx(tx + H, ty + H);
		n.lxm = lidx(tx + H - 1, ty + H);
		n.roff = poff(x0 + tx, y0 + ty);
		return n;
	};
	// stage nodes per plane parity: red 1st (h = 3, two slots), black 1st
	// (h = 2), red 2nd (h = 1)
	S4Node r1n[2][2], b1n[2], r2n[2];
#pragma unroll
	for (int P = 0; P < 2; P++) {
		r1n[P][0] = mknode(tid, 0, 3, P);
		// the red 1st nodes beyond NT go to the last threads (the last wave
		// has no red 2nd node), so no wave does more than three updates in
		// the first phase of a step
		r1n[P][1] = mknode(tid - (2 * NT - S::nodes(3)) + NT, 0, 3, P);
		b1n[P] = mknode(tid, 1, 2, P);
		r2n[P] = mknode(tid, 0, 1, P);
	}
	const bool r1second = tid >= 2 * NT - S::nodes(3), b1ok = tid < S::nodes(2), r2ok = tid < S::nodes(1);
	// the output node (black, 2nd iteration): this thread's tile node
	const int otx = tid % SX, oty = tid / SX;
	const unsigned oli = lidx(otx + H, oty + H), olxm = lidx(otx + H - 1, oty + H);
	const unsigned ooff = (unsigned)((x0 + otx) + (y0 + oty) * TX) * 8u;
	const int oblack0 = (x0 + otx + y0 + oty) & 1;  // black on even planes
	// phi halo fetch: region element i = tid + NT k (row-major, HX wide);
	// the third slot's elements on the last threads (those with the fewer
	// black 1st nodes)
	unsigned foff[3], fli[3];
#pragma unroll
	for (int k = 0; k < 3; k++) {
		int i = k < 2 ? tid + NT * k : tid - (3 * NT - PL) + 2 * NT;
		if (i >= PL || i < 0) i = 0;
		foff[k] = poff(x0 + i % HX - H, y0 + i / HX - H);
		fli[k] = lidx(i % HX, i / HX);
	}
	const bool f2ok = tid >= 3 * NT - PL;
	auto at = [](const double *base, unsigned byteOff) {
		return *(const double *)((const char *)base + byteOff);
	};
#if PINC_MG_S4_PAIRS
	// x pairs of the region (x0 and the region's first column are even, and
	// so is the level's x extent: a pair never straddles the periodic wrap
	// and is 16-B aligned): pair q = tid, and q = tid + 64 on the last wave
	static_assert(PL % 2 == 0 && HX % 2 == 0 && PL / 2 > NT && PL / 2 - NT <= 64, "pair slots");
	typedef s4pair FV;
	constexpr int FN = 2;
	unsigned qoff[2], qli[2];
	const bool q1ok = tid >= NT - (PL / 2 - NT);
#pragma unroll
	for (int k = 0; k < 2; k++) {
		int q = k == 0 ? tid : tid + (PL / 2 - NT);
		if (q >= PL / 2) q = 0;
		const int c = q % (HX / 2), ly = q / (HX / 2);
		qoff[k] = poff(x0 + 2 * c - H, y0 + ly - H);
		qli[k] = lidx(2 * c, ly);  // (x + 1 at qli + HW)
	}
	auto atp = [](const double *base, unsigned byteOff) {
		return *(const s4pair *)((const char *)base + byteOff);
	};
#else
	typedef double FV;
	constexpr int FN = 3;
#endif
	auto plane = [&](const double *a, int q) { return a + (long)wrapi(q, TZ) * sz; };
	// every load below is issued unconditionally (idle lanes and steps past
	// the end load a valid element they do not use): with loads under a
	// branch the compiler's vmcnt waits cannot count the newer loads in
	// flight and wait for the prefetch just issued
#if PINC_MG_S4_PAIRS
	auto fetchP = [&](const double *a, int q, FV *f) {
		const double *b = plane(a, q);
		f[0] = atp(b, qoff[0]);
		f[1] = atp(b, qoff[1]);
	};
	auto putP = [&](double *R, int slot, const FV *f) {
		R[slot * PL + qli[0]] = f[0].x;
		R[slot * PL + qli[0] + HW] = f[0].y;
		if (q1ok) {
			R[slot * PL + qli[1]] = f[1].x;
			R[slot * PL + qli[1] + HW] = f[1].y;
		}
	};
	auto fetch = [&](int q, FV *f) { fetchP(phiIn, q, f); };
	auto putPhi = [&](int slot, const FV *f) { putP(L, slot, f); };
#else
	auto fetch = [&](int q, double *f) {
#if PINC_MG_S4_DIAG & 2
		f[0] = f[1] = f[2] = (double)q;
		return;
#endif
		const double *b = plane(phiIn, q);
		f[0] = at(b, foff[0]);
		f[1] = at(b, foff[1]);
		f[2] = at(b, foff[2]);
	};
	auto putPhi = [&](int slot, const double *f) {
		L[slot * PL + fli[0]] = f[0];
		L[slot * PL + fli[1]] = f[1];
		if (f2ok) L[slot * PL + fli[2]] = f[2];
	};
#endif
#if PINC_MG_S4_RHOLDS && PINC_MG_S4_PAIRS
	auto fetchR = [&](int q, FV *f) { fetchP(rho, q, f); };
	auto putRho = [&](int slot, const FV *f) { putP(Rl, slot, f); };
#elif PINC_MG_S4_RHOLDS
	auto fetchR = [&](int q, double *f) {
#if PINC_MG_S4_DIAG & 1
		f[0] = f[1] = f[2] = (double)q;
		return;
#endif
		const double *b = plane(rho, q);
		f[0] = at(b, foff[0]);
		f[1] = at(b, foff[1]);
		f[2] = at(b, foff[2]);
	};
	auto putRho = [&](int slot, const double *f) {
		Rl[slot * PL + fli[0]] = f[0];
		Rl[slot * PL + fli[1]] = f[1];
		if (f2ok) Rl[slot * PL + fli[2]] = f[2];
	};
#endif
	struct Rho {
		double r1[2], b1, r2, b2;
	};
	// rho of the four stages of step t (t of parity PT)
	auto fetchRho = [&](int t, int PT, Rho &R) {
#if PINC_MG_S4_DIAG & 1
		R.r1[0] = R.r1[1] = R.b1 = R.r2 = R.b2 = (double)t;
		return;
#endif
		const double *b3 = plane(rho, t + 3), *b2p = plane(rho, t + 2), *b0 = plane(rho, t), *bm = plane(rho, t - 2);
		R.r1[0] = at(b3, r1n[PT ^ 1][0].roff);
		R.r1[1] = at(b3, r1n[PT ^ 1][1].roff);
		R.b1 = at(b2p, b1n[PT].roff);
		R.r2 = at(b0, r2n[PT].roff);
		R.b2 = at(bm, ooff);
	};
	// GS update of node n on ring slot SL (neighbours on slots SM, SP).
	// PINC_MG_S4_SPLIT: the second read of each neighbour pair goes through
	// an index the compiler cannot relate to the first (an empty asm), so
	// the pairs stay two ds_read_b64 (2 LDS cycles each) instead of merging
	// into ds_read2_b64 / ds_read2st64_b64 (8 cycles, half the rate)
	auto upd = [&](int SL, int SM, int SP, unsigned li, unsigned lxm, double r) {
#if PINC_MG_S4_SPLIT
		unsigned ixp = lxm + 1, iyp = li + HX, izp = li;
		asm volatile("" : "+v"(ixp));
		asm volatile("" : "+v"(iyp));
		asm volatile("" : "+v"(izp));
		const double xm = L[SL * PL + lxm], xp = L[SL * PL + ixp];
		const double ym = L[SL * PL + li - HX], yp = L[SL * PL + iyp];
		const double zm = L[SM * PL + li], zp = L[SP * PL + izp];
#else
		const double xm = L[SL * PL + lxm], xp = L[SL * PL + lxm + 1];
		const double ym = L[SL * PL + li - HX], yp = L[SL * PL + li + HX];
		const double zm = L[SM * PL + li], zp = L[SP * PL + li];
#endif
		return (1. / 6.) * (xp + xm + yp + ym + zp + zm + r);
	};

	// prologue: phi z0-4 .. z0-2 into LDS, z0-1 into F[1]; rho of the first
	// two steps (z0 is a multiple of 8: plane q sits in slot q & 7)
	constexpr int A = PINC_MG_S4_RHOLDS ? PINC_MG_S4_AHEAD : 2;
	static_assert(A == 2 || A == 3, "24-step unroll: register sets rotate by 2 or 3");
	FV F[A][FN];
	for (int q = z0 - 4; q <= z0 - 2; q++) {
		fetch(q, F[0]);
		putPhi(q & 7, F[0]);
	}
	fetch(z0 - 1, F[1]);
	if (A == 3) fetch(z0, F[2]);
#if PINC_MG_S4_RHOLDS
	// rho planes on the phi ring's schedule: z0-4 .. z0-2 into LDS, z0-1 into
	// G[1]; plane s+6 fetched and s+5 stored at step s
	FV G[A][FN];
	for (int q = z0 - 4; q <= z0 - 2; q++) {
		fetchR(q, G[0]);
		putRho(q & 7, G[0]);
	}
	fetchR(z0 - 1, G[1]);
	if (A == 3) fetchR(z0, G[2]);
#else
	// rho of step k in R[k % 3], loaded two steps ahead; the unroll over 24
	// steps keeps the rotation in register names (a copy of a set just
	// loaded would wait for its loads every step)
	Rho R[3];
	fetchRho(z0 - 6, 0, R[0]);
	fetchRho(z0 - 5, 1, R[1]);
#endif
	__syncthreads();
	const int zEnd = z0 + zPlanes;  // outputs z0 .. zEnd-1
	// steps s = z0-6 .. zEnd+1: zPlanes + 8 of them (a multiple of 24), in
	// blocks of 24 starting at s = 2 (mod 8), so plane s+d sits in slot
	// (2 + k + d) & 7
	for (int s0 = z0 - 6; s0 <= zEnd + 1; s0 += 24) {
#pragma unroll
		for (int k = 0; k < 24; k++) {
			const int s = s0 + k;
			const int P = k & 1;  // parity of s (s0 even)
			auto sl = [&](int d) { return (2 + k + d) & 7; };
#if PINC_MG_S4_RHOLDS
			// rho of a stage's node: its LDS index in the plane's rho slot
			auto rr = [&](int SL, unsigned li) { return Rl[SL * PL + li]; };
			// plane s+4+A into set k % A; the set stored below, plane s+5,
			// was fetched A-1 steps ago into set (k + 1) % A
			fetch(s + 4 + A, F[k % A]);
			fetchR(s + 4 + A, G[k % A]);
#else
			Rho &RA = R[k % 3];
			// two steps ahead of their use (the last step's loads are unused)
			fetch(s + 6, F[P]);
			fetchRho(s + 2, P, R[(k + 2) % 3]);
#endif
			if (s + 3 <= zEnd + 2) {  // red, 1st iteration, plane s+3 (parity P^1)
				const S4Node &a = r1n[P ^ 1][0], &b = r1n[P ^ 1][1];
#if PINC_MG_S4_RHOLDS
				const double ra = rr(sl(3), a.li), rb = rr(sl(3), b.li);
#else
				const double ra = RA.r1[0], rb = RA.r1[1];
#endif
				const double va = upd(sl(3), sl(2), sl(4), a.li, a.lxm, ra);
				double vb = 0;
				if (r1second) vb = upd(sl(3), sl(2), sl(4), b.li, b.lxm, rb);
				L[sl(3) * PL + a.li] = va;
				if (r1second) L[sl(3) * PL + b.li] = vb;
			}
			if (s >= z0 - 1 && s <= zEnd && r2ok) {  // red, 2nd, plane s
				const S4Node &a = r2n[P];
#if PINC_MG_S4_RHOLDS
				L[sl(0) * PL + a.li] = upd(sl(0), sl(-1), sl(1), a.li, a.lxm, rr(sl(0), a.li));
#else
				L[sl(0) * PL + a.li] = upd(sl(0), sl(-1), sl(1), a.li, a.lxm, RA.r2);
#endif
			}
			{  // black, 2nd, plane s-2: out.  Before the first output plane the
			   // store goes to plane z0, rewritten with its value later (the
			   // store is unconditional for the same reason as the loads)
				double v = L[sl(-2) * PL + oli];
#if PINC_MG_S4_RHOLDS
				if (oblack0 ^ P) v = upd(sl(-2), sl(-3), sl(-1), oli, olxm, rr(sl(-2), oli));
#else
				if (oblack0 ^ P) v = upd(sl(-2), sl(-3), sl(-1), oli, olxm, RA.b2);
#endif
				*(double *)((char *)plane(phiOut, s - 2 >= z0 ? s - 2 : z0) + ooff) = v;
			}
			__syncthreads();
			if (s + 2 >= z0 - 2 && s + 2 <= zEnd + 1 && b1ok) {  // black, 1st, plane s+2
				const S4Node &a = b1n[P];
#if PINC_MG_S4_RHOLDS
				L[sl(2) * PL + a.li] = upd(sl(2), sl(1), sl(3), a.li, a.lxm, rr(sl(2), a.li));
#else
				L[sl(2) * PL + a.li] = upd(sl(2), sl(1), sl(3), a.li, a.lxm, RA.b1);
#endif
			}
			// phi s+5 into the slot of s-3 (last read by the black output above)
			putPhi(sl(5), F[(k + 1) % A]);
#if PINC_MG_S4_RHOLDS
			putRho(sl(5), G[(k + 1) % A]);  // (rho s-3: last read by the black output a step ago)
#endif
			__syncthreads();
		}
	}
}

// ------------------------------------------- coarse levels in one launch ---
// Native mode: the V-cycle below level qc (every level with at most
// kCoarseMax points, down to 2 per dimension) runs inside one 1024-thread
// workgroup with all its grids in LDS, replacing ~100 tiny launches per
// cycle.  Same operators and expression order as the per-level kernels:
// GS (mgGS3D form when gs3d, else mgGSND), residual, restriction
// (halfWeight / halfWeightND), prolongation (prol_low), neutralisation after
// each smoothing and of rho.  1-D, 2-D and 3-D (ND).
constexpr int kCoarseMax = 4096;          // points of the top coarse level
constexpr int kCoarseLds = 5500 * 3;      // doubles: phi, rho, res of all levels (132 KB)

struct CoarseArgs {
	int nLevels;
	int T[12][3];
	int nPre, nPost, nCoarse;
	int hw3d;
	int gs3d;
};

__device__ double blk_sum(double v, double *wred) {
	v = wave_sum(v);
	int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	__syncthreads();
	if (lane == 0) wred[w] = v;
	__syncthreads();
	double t = 0;
	for (int q = 0; q < (int)(blockDim.x >> 6); q++) t += wred[q];
	__syncthreads();
	return t;
}

__device__ void blk_neutralize(double *a, long n, double *wred) {
	double t = 0;
	for (long g = threadIdx.x; g < n; g += blockDim.x) t += a[g];
	double mu = blk_sum(t, wred) / (double)n;
	for (long g = threadIdx.x; g < n; g += blockDim.x) a[g] = a[g] - mu;
	__syncthreads();
}

// (the coarse levels hold at most 5500 points: 32-bit index arithmetic)
__device__ __forceinline__ void blk_coords(const Lv &L, long g, int *c) {
	const int gi = (int)g, T0 = L.T[0], T1 = L.T[1];
	c[0] = gi % T0;
	const int r = gi / T0;
	c[1] = r % T1;
	c[2] = r / T1;
}

// one GS update of point c (linear index g) of a coarse level, the
// expression order of mgGS3D / mgGSND
template <int ND>
__device__ __forceinline__ void blk_update(double *phi, const double *rho, const Lv &L, const int *c, long g,
                                           bool gs3d) {
	double v;
	if (ND == 3 && gs3d) {
		double xp = phi[g + nb_up(L, c, 0)], xm = phi[g + nb_dn(L, c, 0)];
		double yp = phi[g + nb_up(L, c, 1)], ym = phi[g + nb_dn(L, c, 1)];
		double zp = phi[g + nb_up(L, c, 2)], zm = phi[g + nb_dn(L, c, 2)];
		v = (1. / 6.) * (xp + xm + yp + ym + zp + zm + rho[g]);
	} else {
		v = 0;
#pragma unroll
		for (int d = 0; d < ND; d++) v += phi[g + nb_up(L, c, d)] + phi[g + nb_dn(L, c, d)];
		v += rho[g];
		v *= 1. / (2 * ND);
	}
	phi[g] = v;
}

// red-black iterations.  Even x extent (every level of a power-of-two
// grid): each colour pass visits only its own points (point 2i + parity of
// row (y, z)); otherwise all points, skipping the other colour.  The
// updates of one colour are independent: the same result either way.
template <int ND>
__device__ void blk_smooth(double *phi, const double *rho, const Lv &L, int nIter, bool gs3d) {
	const int T0 = L.T[0], T1 = L.T[1], n = T0 * T1 * L.T[2];
	const int half = T0 >> 1, nPairs = half * T1 * L.T[2];
	const bool even = (T0 & 1) == 0;
	for (int it = 0; it < nIter; it++) {
		for (int pass = 0; pass < 2; pass++) {
			if (even) {
				for (int q = threadIdx.x; q < nPairs; q += blockDim.x) {
					const int r = q / half, i = q - r * half;
					int c[3];
					c[1] = r % T1;
					c[2] = r / T1;
					c[0] = 2 * i + ((pass + c[1] + c[2]) & 1);
					blk_update<ND>(phi, rho, L, c, (long)c[0] + (long)c[1] * L.s[1] + (long)c[2] * L.s[2], gs3d);
				}
			} else {
				for (int g = threadIdx.x; g < n; g += blockDim.x) {
					int c[3];
					blk_coords(L, g, c);
					if (((c[0] + c[1] + c[2]) & 1) != pass) continue;
					blk_update<ND>(phi, rho, L, c, g, gs3d);
				}
			}
			__syncthreads();
		}
	}
}

struct CLevel {
	Lv L;
	long N;
	double *phi, *rho, *res;
};

// level l's grids inside the LDS block (no dynamically indexed arrays:
// everything is recomputed from the kernel arguments)
template <int ND>
__device__ __forceinline__ CLevel clevel(const CoarseArgs &a, double *lds, int l) {
	CLevel c;
	long off = 0;
	for (int k = 0; k < l; k++) off += 3L * a.T[k][0] * a.T[k][1] * a.T[k][2];
	pinc_lvl_t lp;
	lp.nd = ND;
	lp.T[0] = a.T[l][0];
	lp.T[1] = a.T[l][1];
	lp.T[2] = a.T[l][2];
	c.L = make_lv(lp);
	c.N = (long)lp.T[0] * lp.T[1] * lp.T[2];
	c.phi = lds + off;
	c.rho = lds + off + c.N;
	c.res = lds + off + 2 * c.N;
	return c;
}

// the V-cycle of the LDS levels: level 0 of the block holds rho (and phi = 0)
// on entry and the correction on return (k_mg_coarse, k_mg_solve_small)
template <int ND>
__device__ void coarse_body(const CoarseArgs &a, double *lds, double *wred) {
	const bool gs3d = a.gs3d;
	const int B = a.nLevels - 1;
	for (int l = 0; l < B; l++) {
		CLevel f = clevel<ND>(a, lds, l), c = clevel<ND>(a, lds, l + 1);
		blk_neutralize(f.rho, f.N, wred);
		blk_smooth<ND>(f.phi, f.rho, f.L, a.nPre, gs3d);
		for (long g = threadIdx.x; g < f.N; g += blockDim.x) {
			int q[3];
			blk_coords(f.L, g, q);
			f.res[g] = residual_at<ND>(f.phi, f.rho, f.L, q, g);
		}
		__syncthreads();
		const Lv &F = f.L, &C = c.L;
		for (long gc = threadIdx.x; gc < c.N; gc += blockDim.x) {
			int cc[3], cf[3] = {0, 0, 0};
			blk_coords(C, gc, cc);
			long gf = 0;
#pragma unroll
			for (int d = 0; d < ND; d++) {
				cf[d] = 2 * cc[d];
				gf += (long)cf[d] * F.s[d];
			}
			const double *x = f.res;
			double v;
			if (ND == 3 && a.hw3d) {
				v = (1. / 12.) * (6 * x[gf] + x[gf + nb_up(F, cf, 0)] + x[gf + nb_dn(F, cf, 0)] +
				                  x[gf + nb_up(F, cf, 1)] + x[gf + nb_dn(F, cf, 1)] +
				                  x[gf + nb_up(F, cf, 2)] + x[gf + nb_dn(F, cf, 2)]);
			} else {
				v = (2. * ND) * x[gf];
#pragma unroll
				for (int d = 0; d < ND; d++) v += x[gf + nb_up(F, cf, d)] + x[gf + nb_dn(F, cf, d)];
				v *= 1. / (ND * 4);
			}
			c.rho[gc] = v * 4.0;  // native: coarse h^2 factor (the host path's k_scale order)
			c.phi[gc] = 0.0;      // correction scheme
		}
		__syncthreads();
	}
	{
		CLevel b = clevel<ND>(a, lds, B);
		blk_neutralize(b.rho, b.N, wred);
		blk_smooth<ND>(b.phi, b.rho, b.L, a.nCoarse, gs3d);
		blk_neutralize(b.phi, b.N, wred);
	}
	for (int l = B - 1; l >= 0; l--) {
		CLevel f = clevel<ND>(a, lds, l), c = clevel<ND>(a, lds, l + 1);
		for (long g = threadIdx.x; g < f.N; g += blockDim.x) {
			int cf[3];
			blk_coords(f.L, g, cf);
			f.phi[g] += prol_low<ND, 0>(c.phi, c.L, cf);
		}
		__syncthreads();
		// no neutralisation before the post-smoothing (native mode, round 4):
		// the smoother commutes with adding a constant, the one after it
		// removes the mean
		blk_smooth<ND>(f.phi, f.rho, f.L, a.nPost, gs3d);
		blk_neutralize(f.phi, f.N, wred);
	}
}

template <int ND>
__global__ __launch_bounds__(1024) void k_mg_coarse(const double *__restrict__ rhoIn,
                                                    double *__restrict__ phiOut, CoarseArgs a) {
	__shared__ double lds[kCoarseLds];
	__shared__ double wred[16];
	{
		CLevel t = clevel<ND>(a, lds, 0);
		for (long g = threadIdx.x; g < t.N; g += blockDim.x) {
			t.rho[g] = rhoIn[g];
			t.phi[g] = 0.0;
		}
	}
	__syncthreads();
	coarse_body<ND>(a, lds, wred);
	CLevel t = clevel<ND>(a, lds, 0);
	for (long g = threadIdx.x; g < t.N; g += blockDim.x) phiOut[g] = t.phi[g];
}

// ------------------------------------------ a whole small solve in one CU ---
// Native mode, one rank, a 2-D level 0 of at most kSmallMax points (x extent
// a power of two; C2's 128^2): every cycle of a solve, and the convergence
// test, in one 1024-thread workgroup.  Each thread owns fixed level-0 points
// of alternating colours and holds their rho in registers while it smooths
// them (loaded per smoothing: 16 slots' worth live across the whole cycle
// would spill at 1024 threads); phi lives in LDS
// (colour-major) while it is smoothed, then goes through memory (phi, its own
// buffer; the residual through res) while the LDS holds the coarse solve:
// the V-cycle of levels 1.. (coarse_body), or with multigrid:spectralCoarse
// level 1 solved exactly (below).  The operators and their expression order
// are those of the multi-launch path (k_gs_pass with no shift = blk_update;
// residual_at; k_restrict x 4; prol_low), so in the V-cycle form phi is
// bit-identical to it for the same number of cycles; only the order of the
// norm's sum differs.  This replaces the ~25 launches of each cycle (4-5 us
// each at 128^2) and the host's norm read per cycle by one launch and one
// read per solve.
constexpr int kSmallMax = 16384;
constexpr int kSmallPer = kSmallMax / 1024;
static_assert(kSmallMax <= kCoarseLds, "level 0 in the coarse LDS block");

// multigrid:spectralCoarse in the same workgroup: the level-1 correction
// equation -L phi1 = rho1 on a square n x n level 1 (n a multiple of 16, at
// most 64) solved exactly in LDS through the real orthonormal Fourier basis Q
// of the periodic second difference (columns: DC, cos k, Nyquist, sin k;
// eigenvalue 2 - 2 cos(2 pi k / n) per dimension, DC dropped) -- phi1 =
// Q ((Q^T rho1 Q) / (lam_y + lam_x)) Q^T, four n^3 products on the f64
// matrix cores (v_mfma_f64_16x16x4_f64, one 16 x 16 output tile per wave).
// The same discrete problem as the rocFFT path's (k_spectral_scale's
// symbol), in another rounding.  Matrices in LDS with rows padded to n + 1
// doubles (the operand reads of 16 lanes down a column spread over the
// banks).
typedef double f64x4 __attribute__((ext_vector_type(4)));

// one 16 x 16 tile (rows i0.., columns j0..) of op(A) op(B), K the inner
// extent; lane l returns D[i0 + (l >> 4) + 4 r][j0 + (l & 15)] in element r
template <bool TA, bool TB>
__device__ __forceinline__ f64x4 mm_tile(const double *A, const double *B, int ld, int i0, int j0, int K, int tid) {
	const int lane = tid & 63;
	const int ii = i0 + (lane & 15), jj = j0 + (lane & 15), kl = lane >> 4;
	f64x4 acc = {0.0, 0.0, 0.0, 0.0};
	for (int k0 = 0; k0 < K; k0 += 4) {
		const int kk = k0 + kl;
		const double x = TA ? A[kk * ld + ii] : A[ii * ld + kk];
		const double y = TB ? B[jj * ld + kk] : B[kk * ld + jj];
		acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
	}
	return acc;
}

// D = op(A) op(B) (n x n, ld = n + 1) by the workgroup's waves, a tile per
// wave (tid = threadIdx.x, passed in so the caller controls its hoisting);
// scaled by 1 / (lam[row] + lam[col]) (0 at DC) when lam (LDS) is given
template <bool TA, bool TB>
__device__ __forceinline__ void mm_block(const double *A, const double *B, double *D, int n, const double *lam,
                                         int tid) {
	const int ld = n + 1, nt = n >> 4, w = tid >> 6, lane = tid & 63;
	if (w < nt * nt) {
		const int i0 = (w / nt) << 4, j0 = (w % nt) << 4;
		const f64x4 acc = mm_tile<TA, TB>(A, B, ld, i0, j0, n, tid);
		const int col = j0 + (lane & 15);
#pragma unroll
		for (int r = 0; r < 4; r++) {
			const int row = i0 + (lane >> 4) + 4 * r;
			double v = acc[r];
			if (lam) v = (row == 0 && col == 0) ? 0.0 : v * (1.0 / (lam[row] + lam[col]));
			D[row * ld + col] = v;
		}
	}
	__syncthreads();
}

struct SmallArgs {
	CoarseArgs c;      // levels 1 .. of the solve (c.T[0] = level 1)
	int T0[2];         // level 0 (2-D)
	int lgH;           // log2 of T0 / 2
	int nPre, nPost;   // level-0 smoothing
	int maxCycles;     // stop (with the history) after this many cycles
	double tol;        // stop once the RMS residual is <= tol (or not finite)
};

#ifndef PINC_SMALL_DIAG
#define PINC_SMALL_DIAG 0  // 1: the first cycle's phase times (100 MHz ticks) in out[2..] instead of the history
#endif

// (phi and res not __restrict__: other waves of the workgroup read what a
// wave wrote before a barrier)
template <bool SPEC, int P>
__global__ __launch_bounds__(1024) void k_mg_solve_small2(double *phi, const double *__restrict__ rho, double *res,
                                                          SmallArgs a, double *__restrict__ out,
                                                          const double *__restrict__ basis) {
	static_assert(P % 2 == 0 && P <= kSmallPer, "slots per thread");
	constexpr int ND = 2;
	__shared__ double lds[kCoarseLds];
	__shared__ double wred[16];
	pinc_lvl_t l0;
	l0.nd = ND;
	l0.T[0] = a.T0[0];
	l0.T[1] = a.T0[1];
	l0.T[2] = 1;
	const Lv L = make_lv(l0);
	const int T0 = a.T0[0], T1 = a.T0[1], N0 = T0 * T1, NH = N0 >> 1, H = T0 >> 1;
	const int t = threadIdx.x;
	// slot j of this thread: colour c = j & 1, pair q = t + 1024 k (k = j >> 1)
	// of that colour: row y = q / H, x = 2 (q % H) + ((c + y) & 1).  In LDS
	// level 0 is colour-major, point (x, y) of colour c at c NH + y H + x / 2,
	// so a wave's updates and their neighbour reads are unit-stride.  With H
	// dividing 512 the column q % H = t % H and the x parity do not depend on
	// k, and slot k sits 1024 k above slot 0 in both colour arrays (2048 k in
	// level 0's memory): per colour a handful of per-thread bases, the rest
	// compile-time offsets (no address arithmetic per update but the y wrap)
	const int R = 1024 >> a.lgH;  // rows per slot pair
	// the per-colour bases, recomputed from the thread index at the top of
	// each phase (refresh: the index through an empty asm), so that neither
	// they nor the slots' addresses (5 per slot) stay live across the cycle
	// loop
	int tid = t;
	int y0, xc[2], own[2], xpI[2], xmI[2], ob[2], g0[2];
	auto refresh = [&]() {
		asm volatile("" : "+v"(tid));
		const int i0 = tid & (H - 1);
		y0 = tid >> a.lgH;
#pragma unroll
		for (int c = 0; c < 2; c++) {
			const int x = 2 * i0 + ((c + y0) & 1);
			const int row = (1 - c) * NH + y0 * H;  // row y0 of the other colour
			xc[c] = x;
			own[c] = c * NH + tid;
			xpI[c] = row + (x + 1 < T0 ? (x + 1) >> 1 : 0);
			xmI[c] = row + (x > 0 ? (x - 1) >> 1 : (T0 - 1) >> 1);
			ob[c] = row + (x >> 1);
			g0[c] = x + y0 * T0;
		}
	};
	refresh();
	struct Slot {
		int g, li, x, y;
	};
	auto slot = [&](int j) -> Slot {
		const int c = j & 1, k = j >> 1;
		Slot r;
		r.x = xc[c];
		r.y = y0 + k * R;
		r.g = g0[c] + 2048 * k;
		r.li = own[c] + 1024 * k;
		return r;
	};
	// the four neighbours' LDS indices (other colour): x+1, x-1, y+1, y-1
	auto nbr = [&](const Slot &p, int j, int *o) {
		const int c = j & 1, k = j >> 1;
		const int b = ob[c] + 1024 * k;
		o[0] = xpI[c] + 1024 * k;
		o[1] = xmI[c] + 1024 * k;
		o[2] = p.y + 1 < T1 ? b + H : b - p.y * H;
		o[3] = p.y > 0 ? b - H : b + (T1 - 1) * H;
	};
	auto stamp = [&](int k) {
		if (PINC_SMALL_DIAG && t == 0) out[2 + k] = (double)wall_clock64();
	};
#pragma unroll
	for (int j = 0; j < P; j++) {
		const Slot p = slot(j);
		lds[p.li] = phi[p.g];
		if (j & 1) __builtin_amdgcn_sched_barrier(0);  // 2 slots per batch
	}
	__syncthreads();
	// r of slot j from the phi in LDS (residual_at's expression)
	auto resid = [&](int j, double rj) {
		const Slot p = slot(j);
		int o[4];
		nbr(p, j, o);
		double r = -(2. * ND) * lds[p.li];
		r += lds[o[0]] + lds[o[1]];
		r += lds[o[2]] + lds[o[3]];
		return r + rj;
	};
	// nIter red-black iterations (blk_update's expression: (x+ + x-) +
	// (y+ + y-), + rho, / 4).  The thread's rho is loaded into registers at
	// the start and dies at the end, so the other phases have the whole
	// register budget.
	auto smooth0 = [&](int nIter) {
		refresh();
		double rr[P];
#pragma unroll
		for (int j = 0; j < P; j++) rr[j] = rho[slot(j).g];
		for (int it = 0; it < nIter; it++) {
			for (int pass = 0; pass < 2; pass++) {
				refresh();
				// every read of the pass before its first write (the slots
				// of one colour read only the other colour): the LDS reads
				// of the thread's updates in flight together, 16 at a time
				double v[P / 2];
#pragma unroll
				for (int k = 0; k < P / 2; k++) {
					const int j = 2 * k + pass;
					const Slot p = slot(j);
					int o[4];
					nbr(p, j, o);
					v[k] = 0;
					v[k] += lds[o[0]] + lds[o[1]];
					v[k] += lds[o[2]] + lds[o[3]];
					if ((k & 3) == 3) __builtin_amdgcn_sched_barrier(0);
				}
#pragma unroll
				for (int k = 0; k < P / 2; k++) {
					const int j = 2 * k + pass;
					const Slot p = slot(j);
					double w = v[k] + rr[j];
					w *= 1. / (2 * ND);
					lds[p.li] = w;
				}
				__syncthreads();
			}
		}
	};
	// the residuals in a rolled loop over slot pairs, rho from memory (the
	// residual's reads of every slot unrolled at once need more registers
	// than the workgroup size allows at 16 slots): tail = 1 stores them and
	// phi to memory (the restriction's input), tail = 2 returns the sum of
	// their squares
	auto residuals = [&](int tail) -> double {
		double s2 = 0;
		refresh();
#pragma unroll 1
		for (int k = 0; k < P / 2; k++) {
#pragma unroll
			for (int c = 0; c < 2; c++) {
				const int j = 2 * k + c;
				const Slot p = slot(j);
				const double r = resid(j, rho[p.g]);
				if (tail == 1) {
					res[p.g] = r;
					phi[p.g] = lds[p.li];
				} else {
					s2 += r * r;
				}
			}
		}
		return s2;
	};
	const CLevel c1 = clevel<ND>(a.c, lds, 0);
	int cyc = 0;
	double bar = 0;
	for (;;) {
		if (cyc == 0) stamp(0);
		smooth0(a.nPre);
		if (cyc == 0) stamp(1);
		// the residual and phi of the own points to memory
		residuals(1);
		__syncthreads();
		if (cyc == 0) stamp(2);
		if constexpr (SPEC) {
			// the restricted residual (x 4) into R, Q beside it, then the
			// exact level-1 solve; phi1 ends in R
			const int n = c1.L.T[0], ld = n + 1;
			double *R = lds, *Tm = lds + n * ld, *Qs = lds + 2 * n * ld;
			refresh();
			for (int e = tid; e < n * n + n; e += 1024)  // Q, then lambda after its n padded rows
				Qs[e < n * n ? (e / n) * ld + e % n : n * ld + e - n * n] = basis[e];
			for (int gc = tid; gc < n * n; gc += 1024) {
				int cf[3] = {2 * (gc % n), 2 * (gc / n), 0};
				const long gf = cf[0] + (long)cf[1] * L.s[1];
				double v = (2. * ND) * res[gf];
#pragma unroll
				for (int d = 0; d < ND; d++) v += res[gf + nb_up(L, cf, d)] + res[gf + nb_dn(L, cf, d)];
				v *= 1. / (ND * 4);
				R[(gc / n) * ld + gc % n] = v * 4.0;
			}
			__syncthreads();
			if (cyc == 0) stamp(3);
			refresh();
			const double *lam = Qs + n * ld;
			mm_block<false, false>(R, Qs, Tm, n, nullptr, tid);  // R Q
			mm_block<true, false>(Qs, Tm, R, n, lam, tid);       // Q^T (R Q), / lambda
			mm_block<false, true>(R, Qs, Tm, n, nullptr, tid);   // . Q^T
			mm_block<false, false>(Qs, Tm, R, n, nullptr, tid);  // Q (.)
			if (cyc == 0) stamp(4);
			Lv C = c1.L;
			C.s[1] = ld;
			refresh();
#pragma unroll
			for (int j = 0; j < P; j++) {
				const Slot p = slot(j);
				int c[3] = {p.x, p.y, 0};
				phi[p.g] = phi[p.g] + prol_low<ND, 0>(R, C, c);
				if (j & 1) __builtin_amdgcn_sched_barrier(0);
			}
		} else {
			// restriction (k_mg_coarse's expression, x 4) into the coarse block
			refresh();
			for (int gc = tid; gc < c1.N; gc += 1024) {
				int cc[3], cf[3] = {0, 0, 0};
				blk_coords(c1.L, gc, cc);
				long gf = 0;
#pragma unroll
				for (int d = 0; d < ND; d++) {
					cf[d] = 2 * cc[d];
					gf += (long)cf[d] * L.s[d];
				}
				double v = (2. * ND) * res[gf];
#pragma unroll
				for (int d = 0; d < ND; d++) v += res[gf + nb_up(L, cf, d)] + res[gf + nb_dn(L, cf, d)];
				v *= 1. / (ND * 4);
				c1.rho[gc] = v * 4.0;
				c1.phi[gc] = 0.0;
			}
			__syncthreads();
			if (cyc == 0) stamp(3);
			coarse_body<ND>(a.c, lds, wred);
			if (cyc == 0) stamp(4);
			// phi += prolongated level-1 correction, through memory
			refresh();
#pragma unroll
			for (int j = 0; j < P; j++) {
				const Slot p = slot(j);
				int c[3] = {p.x, p.y, 0};
				phi[p.g] = phi[p.g] + prol_low<ND, 0>(c1.phi, c1.L, c);
				if (j & 1) __builtin_amdgcn_sched_barrier(0);
			}
		}
		__syncthreads();
		if (cyc == 0) stamp(5);
		refresh();
#pragma unroll
		for (int j = 0; j < P; j++) {
			const Slot p = slot(j);
			lds[p.li] = phi[p.g];
			if (j & 1) __builtin_amdgcn_sched_barrier(0);
		}
		__syncthreads();
		if (cyc == 0) stamp(6);
		smooth0(a.nPost);
		if (cyc == 0) stamp(7);
		// the RMS residual of the cycle
		const double s2 = residuals(2);
		// mgSolve's test: sqrt(sum / N0) > tol continues (a NaN or an
		// infinity stops, for the host to report)
		bar = sqrt(blk_sum(s2, wred) / (double)N0);
		if (cyc == 0) stamp(8);
		if (!PINC_SMALL_DIAG && t == 0 && cyc < 60) out[2 + cyc] = bar;
		cyc++;
		if (!(bar > a.tol) || isinf(bar) || cyc >= a.maxCycles) break;
	}
	refresh();
#pragma unroll
	for (int j = 0; j < P; j++) {
		const Slot p = slot(j);
		phi[p.g] = lds[p.li];
		if (j & 1) __builtin_amdgcn_sched_barrier(0);
	}
	if (t == 0) {
		out[0] = (double)cyc;
		out[1] = bar;
	}
}

// ----------------------------------------------- sharded level 0 (z-slabs) ---
// Native mode with several ranks: level 0 lives as this
// rank's z-slab extended by hz halo planes on each side, x/y periodic, the
// slab dimension not (its halo planes are in memory).  Level 1 is global.
// Restriction of the slab's residual into this rank's level-1 planes, and
// bilinear prolongation of the global level-1 correction into every plane
// of the extended slab, with the arithmetic of k_restrict / k_prolong_add.

// residual on planes [zlo, zhi) of the extended slab (z neighbours direct);
// SUMSQ: block partials of its square instead of storing it
template <bool SUMSQ>
__global__ __launch_bounds__(kThreads) void k_residual_slab(double *__restrict__ out, const double *__restrict__ phi,
                                                            const double *__restrict__ rho, pinc_lvl_t Lp, int zlo,
                                                            int zhi) {
	__shared__ double red[kThreads / 64];
	Lv L = make_lv(Lp);
	const long ps = L.s[2];
	const long n = ps * (zhi - zlo);
	double acc = 0.;
	const Walk w = point_walk(n);
	for (long q = w.g0; q < w.g1; q += w.step) {
		const long g = (long)zlo * ps + q;
		int c[3];
		{  // 32-bit index arithmetic (levels hold < 2^31 points, checked on the host)
			const unsigned u = (unsigned)g, t0 = (unsigned)L.T[0], t1 = (unsigned)L.T[1];
			const unsigned r = u / t0;
			c[0] = (int)(u - r * t0);
			c[1] = (int)(r % t1);
			c[2] = (int)(r / t1);
		}
		double v = -6. * phi[g];
		v += phi[g + nb_up(L, c, 0)] + phi[g + nb_dn(L, c, 0)] + phi[g + nb_up(L, c, 1)] + phi[g + nb_dn(L, c, 1)] +
		     phi[g + ps] + phi[g - ps];
		v = v + rho[g];
		if (SUMSQ) acc += v * v;
		else out[g] = v;
	}
	if (SUMSQ) {
		double t = block_sum(acc, red);
		if (threadIdx.x == 0) out[blockIdx.x] = t;
	}
}

// coarse (x, y, z) of this rank's level-1 planes <- fine (2x, 2y, zf0 + 2z)
// of the extended slab, halfWeight (HW3D) or halfWeightND, times 4 (native)
template <bool HW3D>
__global__ void k_restrict_slab(const double *__restrict__ fine, pinc_lvl_t Lfp, int zf0,
                                double *__restrict__ coarse, pinc_lvl_t Lcp) {
	Lv F = make_lv(Lfp), C = make_lv(Lcp);
	const long ps = F.s[2];
	const long n = (long)C.T[0] * C.T[1] * C.T[2];
	const Walk w = point_walk(n);
	for (long gc = w.g0; gc < w.g1; gc += w.step) {
		int cc[3];
		{  // 32-bit index arithmetic (levels hold < 2^31 points, checked on the host)
			const unsigned u = (unsigned)gc, t0 = (unsigned)C.T[0], t1 = (unsigned)C.T[1];
			const unsigned r = u / t0;
			cc[0] = (int)(u - r * t0);
			cc[1] = (int)(r % t1);
			cc[2] = (int)(r / t1);
		}
		int cf[3] = {2 * cc[0], 2 * cc[1], zf0 + 2 * cc[2]};
		const long gf = (long)cf[0] + (long)cf[1] * F.s[1] + (long)cf[2] * ps;
		double v;
		if (HW3D) {
			v = (1. / 12.) * (6 * fine[gf] + fine[gf + nb_up(F, cf, 0)] + fine[gf + nb_dn(F, cf, 0)] +
			                  fine[gf + nb_up(F, cf, 1)] + fine[gf + nb_dn(F, cf, 1)] + fine[gf + ps] + fine[gf - ps]);
		} else {
			v = 6. * fine[gf];
			v += fine[gf + nb_up(F, cf, 0)] + fine[gf + nb_dn(F, cf, 0)];
			v += fine[gf + nb_up(F, cf, 1)] + fine[gf + nb_dn(F, cf, 1)];
			v += fine[gf + ps] + fine[gf - ps];
			v *= 1. / 12.;
		}
		coarse[gc] = v * 4.0;
	}
}

// every plane of the extended slab += prolongated global level-1 correction;
// plane zl of the slab is global plane (z0 + zl) mod Tz
__global__ void k_prolong_add_slab(double *__restrict__ phiX, pinc_lvl_t Lxp, int z0, int Tz,
                                   const double *__restrict__ phiC, pinc_lvl_t Lcp) {
	Lv X = make_lv(Lxp), C = make_lv(Lcp);
	const long n = (long)X.T[0] * X.T[1] * X.T[2];
	const Walk w = point_walk(n);
	for (long g = w.g0; g < w.g1; g += w.step) {
		int cf[3];
		cf[0] = (int)(g % X.T[0]);
		long r = g / X.T[0];
		cf[1] = (int)(r % X.T[1]);
		int z = z0 + (int)(r / X.T[1]);
		z %= Tz;
		if (z < 0) z += Tz;
		cf[2] = z;
		phiX[g] += prol_low<3, 0>(phiC, C, cf);
	}
}

// the owned planes [hz, hz + nz) of the extended slab += prolongated
// correction of this rank's own level-1 planes (phiCx: those planes with one
// halo plane on each side).  The owned slab starts at an even global plane,
// so fine plane hz + k sits at plane k + 2 of the frame whose coarse plane 0
// is phiCx's lower halo plane: the same parities, the same prol_low
// expression, and every coarse plane it reads lies in phiCx (k + 2 in
// [2, nz + 2) reads coarse planes 1 .. nz/2 + 1).
__global__ void k_prolong_add_own(double *__restrict__ phiX, pinc_lvl_t Lxp, int hz, int nz,
                                  const double *__restrict__ phiCx, pinc_lvl_t Lcp) {
	Lv X = make_lv(Lxp), C = make_lv(Lcp);
	const long n = (long)X.T[0] * X.T[1] * nz;
	const Walk w = point_walk(n);
	for (long q = w.g0; q < w.g1; q += w.step) {
		int cf[3];
		{  // 32-bit index arithmetic (levels hold < 2^31 points, checked on the host)
			const unsigned u = (unsigned)q, t0 = (unsigned)X.T[0], t1 = (unsigned)X.T[1];
			const unsigned r = u / t0;
			cf[0] = (int)(u - r * t0);
			cf[1] = (int)(r % t1);
			cf[2] = (int)(r / t1) + 2;
		}
		phiX[(long)hz * X.s[2] + q] += prol_low<3, 0>(phiCx, C, cf);
	}
}

// ------------------------------------------ level-0 transfers, 3-D (round 4)
// The three point stencils around the coarse correction, restructured so
// that each thread does the work of a whole coarse cell and no point index is
// divided per fine point; each value is the same expression as before, so the
// results are bit-identical to k_residual + k_restrict (+ the native x4) and
// to k_prolong_add.
//
// Restricted residual: coarse point c gets the half-weight restriction
// (mgHalfRestrict3D, multigrid.c:844-911, or the ND form) of the fine
// residual (mgResidual, multigrid.c:1385-1403) at its fine point 2c and the
// six neighbours, the residual computed on the fly (residual_at's order), so
// the fine residual is never written and read back; times `scale` (4 in
// native mode: exact, a power of two).
template <bool HW3D>
__global__ __launch_bounds__(kThreads) void k_resid_restrict3(const double *__restrict__ phi,
                                                              const double *__restrict__ rho,
                                                              double *__restrict__ coarse, pinc_lvl_t Lcp,
                                                              double scale) {
	pinc_lvl_t Lfp = Lcp;
	for (int d = 0; d < 3; d++) Lfp.T[d] = 2 * Lcp.T[d];
	const Lv F = make_lv(Lfp);
	const unsigned CX = Lcp.T[0], CY = Lcp.T[1];
	const unsigned n = CX * CY * (unsigned)Lcp.T[2];
	for (unsigned gc = blockIdx.x * blockDim.x + threadIdx.x; gc < n; gc += gridDim.x * blockDim.x) {
		const unsigned r = gc / CX;
		int cf[3] = {2 * (int)(gc - r * CX), 2 * (int)(r % CY), 2 * (int)(r / CY)};
		const long gf = (long)cf[0] + cf[1] * F.s[1] + cf[2] * F.s[2];
		auto res_nb = [&](int d, int up) {
			int c[3] = {cf[0], cf[1], cf[2]};
			const long o = up ? nb_up(F, cf, d) : nb_dn(F, cf, d);
			c[d] = up ? (cf[d] + 1 < F.T[d] ? cf[d] + 1 : 0) : (cf[d] > 0 ? cf[d] - 1 : F.T[d] - 1);
			return residual_at<3>(phi, rho, F, c, gf + o);
		};
		const double f0 = residual_at<3>(phi, rho, F, cf, gf);
		const double xp = res_nb(0, 1), xm = res_nb(0, 0), yp = res_nb(1, 1), ym = res_nb(1, 0);
		const double zp = res_nb(2, 1), zm = res_nb(2, 0);
		double v;
		if (HW3D) {
			v = (1. / 12.) * (6 * f0 + xp + xm + yp + ym + zp + zm);
		} else {
			v = (2. * 3) * f0;
			v += xp + xm;
			v += yp + ym;
			v += zp + zm;
			v *= 1. / (3 * 4);
		}
		coarse[gc] = v * scale;
	}
}

// k_resid_restrict3 with the fine values read as 16-B x pairs: a coarse
// point's seven residuals need phi on 19 pairs of rows around its fine point
// and rho on 6, instead of 56 single loads.  Each residual is residual_at's
// expression, the restriction the same sum: bit-identical.  Fine x extent
// even and 16-B aligned arrays (the launcher checks).
template <bool HW3D>
__global__ __launch_bounds__(kThreads) void k_resid_restrict3p(const double *__restrict__ phi,
                                                               const double *__restrict__ rho,
                                                               double *__restrict__ coarse, pinc_lvl_t Lcp,
                                                               double scale) {
	const int FX = 2 * Lcp.T[0], FY = 2 * Lcp.T[1], FZ = 2 * Lcp.T[2];
	const long sy = FX, sz = (long)FX * FY;
	const unsigned CX = Lcp.T[0], CY = Lcp.T[1];
	const unsigned n = CX * CY * (unsigned)Lcp.T[2];
	for (unsigned gc = blockIdx.x * blockDim.x + threadIdx.x; gc < n; gc += gridDim.x * blockDim.x) {
		const unsigned r = gc / CX;
		const int X = 2 * (int)(gc - r * CX), Y = 2 * (int)(r % CY), Z = 2 * (int)(r / CY);
		auto wy = [&](int y) { return (long)(y < 0 ? y + FY : (y >= FY ? y - FY : y)) * sy; };
		auto wz = [&](int z) { return (long)(z < 0 ? z + FZ : (z >= FZ ? z - FZ : z)) * sz; };
		const int xm2 = X >= 2 ? X - 2 : X - 2 + FX, xp2 = X + 2 < FX ? X + 2 : X + 2 - FX;
		auto pr = [](const double *a, long o) { return *reinterpret_cast<const double2 *>(a + o); };
		// rows by (dy, dz); x pairs at X-2 (.y = X-1), X (.x = X, .y = X+1), X+2 (.x)
		const long r00 = wy(Y) + wz(Z);
		const double2 c_m = pr(phi, r00 + xm2), c_0 = pr(phi, r00 + X), c_p = pr(phi, r00 + xp2);
		const long ryp = wy(Y + 1) + wz(Z), rym = wy(Y - 1) + wz(Z);
		const long rzp = wy(Y) + wz(Z + 1), rzm = wy(Y) + wz(Z - 1);
		const double2 yp_m = pr(phi, ryp + xm2), yp_0 = pr(phi, ryp + X);
		const double2 ym_m = pr(phi, rym + xm2), ym_0 = pr(phi, rym + X);
		const double2 zp_m = pr(phi, rzp + xm2), zp_0 = pr(phi, rzp + X);
		const double2 zm_m = pr(phi, rzm + xm2), zm_0 = pr(phi, rzm + X);
		const double y2p = pr(phi, wy(Y + 2) + wz(Z) + X).x, y2m = pr(phi, wy(Y - 2) + wz(Z) + X).x;
		const double z2p = pr(phi, wy(Y) + wz(Z + 2) + X).x, z2m = pr(phi, wy(Y) + wz(Z - 2) + X).x;
		const double ypzp = pr(phi, wy(Y + 1) + wz(Z + 1) + X).x, ypzm = pr(phi, wy(Y + 1) + wz(Z - 1) + X).x;
		const double ymzp = pr(phi, wy(Y - 1) + wz(Z + 1) + X).x, ymzm = pr(phi, wy(Y - 1) + wz(Z - 1) + X).x;
		const double2 q_m = pr(rho, r00 + xm2), q_0 = pr(rho, r00 + X);
		const double q_yp = pr(rho, ryp + X).x, q_ym = pr(rho, rym + X).x;
		const double q_zp = pr(rho, rzp + X).x, q_zm = pr(rho, rzm + X).x;
		// residual_at<3>: -6 phi + (x+ + x- + y+ + y- + z+ + z-) + rho
		auto res = [](double c, double xp, double xm, double yp, double ym, double zp, double zm, double q) {
			double v = -6. * c;
			v += xp + xm + yp + ym + zp + zm;
			return v + q;
		};
		const double f0 = res(c_0.x, c_0.y, c_m.y, yp_0.x, ym_0.x, zp_0.x, zm_0.x, q_0.x);
		const double xp = res(c_0.y, c_p.x, c_0.x, yp_0.y, ym_0.y, zp_0.y, zm_0.y, q_0.y);
		const double xm = res(c_m.y, c_0.x, c_m.x, yp_m.y, ym_m.y, zp_m.y, zm_m.y, q_m.y);
		const double yp = res(yp_0.x, yp_0.y, yp_m.y, y2p, c_0.x, ypzp, ypzm, q_yp);
		const double ym = res(ym_0.x, ym_0.y, ym_m.y, c_0.x, y2m, ymzp, ymzm, q_ym);
		const double zp = res(zp_0.x, zp_0.y, zp_m.y, ypzp, ymzp, z2p, c_0.x, q_zp);
		const double zm = res(zm_0.x, zm_0.y, zm_m.y, ypzm, ymzm, c_0.x, z2m, q_zm);
		double v;
		if (HW3D) {
			v = (1. / 12.) * (6 * f0 + xp + xm + yp + ym + zp + zm);
		} else {
			v = (2. * 3) * f0;
			v += xp + xm;
			v += yp + ym;
			v += zp + zm;
			v *= 1. / (3 * 4);
		}
		coarse[gc] = v * scale;
	}
}

// phi_f += P(phi_c) (mgBilinProl3D + gAddTo): one thread per coarse cell
// writes its 2 x 2 x 2 fine points (x pairs as 16-byte accesses) from the 8
// coarse corner values, each point with prol_low's nesting (x outermost, z
// innermost; 0.5 * (a + b) per odd dimension).
__global__ __launch_bounds__(kThreads) void k_prolong_add3c(double *__restrict__ phiF,
                                                            const double *__restrict__ phiC, pinc_lvl_t Lcp) {
	const unsigned CX = Lcp.T[0], CY = Lcp.T[1], CZ = Lcp.T[2];
	const long sy = (long)CX, sz = (long)CX * CY;
	const long fx = 2L * CX, fxy = fx * 2L * CY;
	const unsigned n = CX * CY * CZ;
	for (unsigned gc = blockIdx.x * blockDim.x + threadIdx.x; gc < n; gc += gridDim.x * blockDim.x) {
		const unsigned r = gc / CX;
		const int cx = (int)(gc - r * CX), cy = (int)(r % CY), cz = (int)(r / CY);
		const int cx1 = cx + 1 < (int)CX ? cx + 1 : 0, cy1 = cy + 1 < (int)CY ? cy + 1 : 0;
		const int cz1 = cz + 1 < (int)CZ ? cz + 1 : 0;
		double c[2][2][2];  // [dx][dy][dz]
		const int xs[2] = {cx, cx1}, ys[2] = {cy, cy1}, zs[2] = {cz, cz1};
#pragma unroll
		for (int a = 0; a < 2; a++)
#pragma unroll
			for (int b = 0; b < 2; b++)
#pragma unroll
				for (int e = 0; e < 2; e++) c[a][b][e] = phiC[xs[a] + ys[b] * sy + zs[e] * sz];
#pragma unroll
		for (int k = 0; k < 2; k++) {
#pragma unroll
			for (int j = 0; j < 2; j++) {
				double zv[2][2];  // [dx][dy]: z step
#pragma unroll
				for (int a = 0; a < 2; a++)
#pragma unroll
					for (int b = 0; b < 2; b++) zv[a][b] = k ? 0.5 * (c[a][b][0] + c[a][b][1]) : c[a][b][0];
				double yv[2];
#pragma unroll
				for (int a = 0; a < 2; a++) yv[a] = j ? 0.5 * (zv[a][0] + zv[a][1]) : zv[a][0];
				const double v0 = yv[0], v1 = 0.5 * (yv[0] + yv[1]);
				double2 *f = reinterpret_cast<double2 *>(phiF + 2L * cx + (2L * cy + j) * fx + (2L * cz + k) * fxy);
				double2 t = *f;
				t.x += v0;
				t.y += v1;
				*f = t;
			}
		}
	}
}

}  // namespace

extern "C" int pinc_hip_resid_restrict(const double *phi, const double *rho, double *coarse, pinc_lvl_t Lc,
                                       int hw3d, double scale, void *stream) {
	if (Lc.nd != 3) return set_error(hipErrorInvalidValue, "resid_restrict: 3-D levels only");
	if (8 * npts(Lc) >= (1L << 31)) return set_error(hipErrorInvalidValue, "resid_restrict: level too large");
	hipStream_t st = (hipStream_t)stream;
	const unsigned nb = blocks_for(npts(Lc));
	const bool pairs = PINC_MG_RR_PAIRS &&
	                   !((reinterpret_cast<unsigned long>(phi) | reinterpret_cast<unsigned long>(rho)) & 15);
	if (pairs && hw3d)
		hipLaunchKernelGGL(k_resid_restrict3p<true>, dim3(nb), dim3(kThreads), 0, st, phi, rho, coarse, Lc, scale);
	else if (pairs)
		hipLaunchKernelGGL(k_resid_restrict3p<false>, dim3(nb), dim3(kThreads), 0, st, phi, rho, coarse, Lc, scale);
	else if (hw3d)
		hipLaunchKernelGGL(k_resid_restrict3<true>, dim3(nb), dim3(kThreads), 0, st, phi, rho, coarse, Lc, scale);
	else hipLaunchKernelGGL(k_resid_restrict3<false>, dim3(nb), dim3(kThreads), 0, st, phi, rho, coarse, Lc, scale);
	return check_launch("resid_restrict");
}

extern "C" int pinc_hip_prolong_add3(double *phiF, const double *phiC, pinc_lvl_t Lc, void *stream) {
	if (Lc.nd != 3) return set_error(hipErrorInvalidValue, "prolong_add3: 3-D levels only");
	if (8 * npts(Lc) >= (1L << 31)) return set_error(hipErrorInvalidValue, "prolong_add3: level too large");
	if (reinterpret_cast<unsigned long>(phiF) & 15)
		return set_error(hipErrorInvalidValue, "prolong_add3: fine grid not 16-byte aligned");
	hipLaunchKernelGGL(k_prolong_add3c, dim3(blocks_for(npts(Lc))), dim3(kThreads), 0, (hipStream_t)stream, phiF,
	                   phiC, Lc);
	return check_launch("prolong_add3");
}

extern "C" int pinc_hip_gs_pass(double *phi, const double *rho, pinc_lvl_t L, int pass, int nd3,
                                const double *muPrev, double *partial, int *nBlocks, void *stream) {
	if (npts(L) >= (1L << 31)) return set_error(hipErrorInvalidValue, "gs_pass: level too large for 32-bit indexing");
	long nPairs = npts(L) / 2;
	unsigned nb = blocks_for(nPairs);
	*nBlocks = (int)nb;
	hipStream_t st = (hipStream_t)stream;
	if (L.nd == 3 && nd3)
		hipLaunchKernelGGL((k_gs_pass<3, true>), dim3(nb), dim3(kThreads), 0, st, phi, rho, L, pass, muPrev, partial);
	else if (L.nd == 3)
		hipLaunchKernelGGL((k_gs_pass<3, false>), dim3(nb), dim3(kThreads), 0, st, phi, rho, L, pass, muPrev, partial);
	else if (L.nd == 2)
		hipLaunchKernelGGL((k_gs_pass<2, false>), dim3(nb), dim3(kThreads), 0, st, phi, rho, L, pass, muPrev, partial);
	else
		hipLaunchKernelGGL((k_gs_pass<1, false>), dim3(nb), dim3(kThreads), 0, st, phi, rho, L, pass, muPrev, partial);
	return check_launch("gs_pass");
}

extern "C" int pinc_hip_gs_materialize(double *phi, pinc_lvl_t L, int lastPass, const double *muA,
                                       const double *muB, void *stream) {
	if (npts(L) >= (1L << 31)) return set_error(hipErrorInvalidValue, "gs_materialize: level too large for 32-bit indexing");
	hipLaunchKernelGGL(k_gs_materialize, dim3(blocks_for(npts(L))), dim3(kThreads), 0,
	                   (hipStream_t)stream, phi, L, lastPass, muA, muB);
	return check_launch("gs_materialize");
}

extern "C" int pinc_hip_residual(double *res, const double *phi, const double *rho, pinc_lvl_t L,
                                 void *stream) {
	if (npts(L) >= (1L << 31)) return set_error(hipErrorInvalidValue, "residual: level too large for 32-bit indexing");
	hipStream_t st = (hipStream_t)stream;
	unsigned nb = blocks_for(npts(L));
	if (L.nd == 3) hipLaunchKernelGGL(k_residual<3>, dim3(nb), dim3(kThreads), 0, st, res, phi, rho, L);
	else if (L.nd == 2) hipLaunchKernelGGL(k_residual<2>, dim3(nb), dim3(kThreads), 0, st, res, phi, rho, L);
	else hipLaunchKernelGGL(k_residual<1>, dim3(nb), dim3(kThreads), 0, st, res, phi, rho, L);
	return check_launch("residual");
}

extern "C" int pinc_hip_residual_sumsq(const double *phi, const double *rho, pinc_lvl_t L,
                                       double *partial, int *nBlocks, void *stream) {
	if (npts(L) >= (1L << 31)) return set_error(hipErrorInvalidValue, "residual_sumsq: level too large for 32-bit indexing");
	hipStream_t st = (hipStream_t)stream;
	unsigned nb = blocks_for(npts(L));
	*nBlocks = (int)nb;
	if (L.nd == 3 && PINC_MG_NORM_PAIRS && L.T[0] % 2 == 0 &&
	    !((reinterpret_cast<unsigned long>(phi) | reinterpret_cast<unsigned long>(rho)) & 15)) {
		nb = blocks_for(npts(L) / 2);
		*nBlocks = (int)nb;
		hipLaunchKernelGGL(k_residual_sumsq3p, dim3(nb), dim3(kThreads), 0, st, phi, rho, L, partial);
	} else if (L.nd == 3) hipLaunchKernelGGL(k_residual_sumsq<3>, dim3(nb), dim3(kThreads), 0, st, phi, rho, L, partial);
	else if (L.nd == 2) hipLaunchKernelGGL(k_residual_sumsq<2>, dim3(nb), dim3(kThreads), 0, st, phi, rho, L, partial);
	else hipLaunchKernelGGL(k_residual_sumsq<1>, dim3(nb), dim3(kThreads), 0, st, phi, rho, L, partial);
	return check_launch("residual_sumsq");
}

extern "C" int pinc_hip_restrict(const double *fine, double *coarse, pinc_lvl_t Lc, int nd3, void *stream) {
	if (npts(Lc) >= (1L << 31)) return set_error(hipErrorInvalidValue, "restrict: level too large for 32-bit indexing");
	hipStream_t st = (hipStream_t)stream;
	unsigned nb = blocks_for(npts(Lc));
	if (Lc.nd == 3 && nd3) hipLaunchKernelGGL((k_restrict<3, true>), dim3(nb), dim3(kThreads), 0, st, fine, coarse, Lc);
	else if (Lc.nd == 3) hipLaunchKernelGGL((k_restrict<3, false>), dim3(nb), dim3(kThreads), 0, st, fine, coarse, Lc);
	else if (Lc.nd == 2) hipLaunchKernelGGL((k_restrict<2, false>), dim3(nb), dim3(kThreads), 0, st, fine, coarse, Lc);
	else hipLaunchKernelGGL((k_restrict<1, false>), dim3(nb), dim3(kThreads), 0, st, fine, coarse, Lc);
	return check_launch("restrict");
}

extern "C" int pinc_hip_prolong_add(double *phiF, const double *phiC, pinc_lvl_t Lf, void *stream) {
	if (npts(Lf) >= (1L << 31)) return set_error(hipErrorInvalidValue, "prolong_add: level too large for 32-bit indexing");
	hipStream_t st = (hipStream_t)stream;
	unsigned nb = blocks_for(npts(Lf));
	if (Lf.nd == 3) hipLaunchKernelGGL(k_prolong_add<3>, dim3(nb), dim3(kThreads), 0, st, phiF, phiC, Lf);
	else if (Lf.nd == 2) hipLaunchKernelGGL(k_prolong_add<2>, dim3(nb), dim3(kThreads), 0, st, phiF, phiC, Lf);
	else hipLaunchKernelGGL(k_prolong_add<1>, dim3(nb), dim3(kThreads), 0, st, phiF, phiC, Lf);
	return check_launch("prolong_add");
}

extern "C" int pinc_hip_gs_sweep(const double *phiIn, double *phiOut, const double *rho, pinc_lvl_t L,
                                 void *stream) {
	// 32x8 column tiles (measured best at 256^3: 0.115 ms against 0.165 ms
	// for k_gs_sweep), planes per workgroup chosen for >= 1024 workgroups
	if (L.nd == 3 && L.T[0] % 32 == 0 && L.T[1] % 8 == 0 && L.T[2] % 16 == 0) {
		long cols = (long)(L.T[0] / 32) * (L.T[1] / 8);
		int zp = 16;
		for (int z = 64; z > 16; z /= 2)
			if (L.T[2] % z == 0 && cols * (L.T[2] / z) >= 1024) {
				zp = z;
				break;
			}
		unsigned nb = (unsigned)(cols * (L.T[2] / zp));
		hipLaunchKernelGGL((k_gs_sweep2<32, 8, 256>), dim3(nb), dim3(256), 0, (hipStream_t)stream, phiIn, phiOut, rho,
		                   L, zp);
		return check_launch("gs_sweep2");
	}
	if (L.nd != 3 || L.T[0] % kSwT || L.T[1] % kSwT || L.T[2] % kSwZ)
		return set_error(hipErrorInvalidValue, "gs_sweep: level not a multiple of the 16x16x16 tile");
	unsigned nb = (unsigned)((L.T[0] / kSwT) * (L.T[1] / kSwT) * (L.T[2] / kSwZ));
	hipLaunchKernelGGL(k_gs_sweep, dim3(nb), dim3(256), 0, (hipStream_t)stream, phiIn, phiOut, rho, L);
	return check_launch("gs_sweep");
}

extern "C" int pinc_hip_gs_sweep2x(const double *phiIn, double *phiOut, const double *rho, pinc_lvl_t L,
                                   void *stream) {
	// two iterations per launch; 32x8 column tiles, planes per workgroup for
	// >= 1024 workgroups where the level allows (at least 16)
	if (L.nd != 3 || L.T[0] % 32 || L.T[1] % 8 || L.T[2] % 16)
		return set_error(hipErrorInvalidValue, "gs_sweep2x: level not a multiple of the 32x8x16 tile");
	if ((reinterpret_cast<unsigned long>(phiIn) | reinterpret_cast<unsigned long>(phiOut) |
	     reinterpret_cast<unsigned long>(rho)) & 15)
		return set_error(hipErrorInvalidValue, "gs_sweep2x: arrays not 16-byte aligned (x-pair fetches)");
	long cols = (long)(L.T[0] / 32) * (L.T[1] / 8);
	int zp = 16;
	for (int z = 64; z > 16; z /= 2)
		if (L.T[2] % z == 0 && cols * (L.T[2] / z) >= 1024 && (!PINC_MG_SWEEP4C || (z + 8) % 24 == 0)) {
			zp = z;  // k_gs_sweep4c marches in blocks of 24 steps: zPlanes + 8 = 24 m
			break;
		}
	unsigned nb = (unsigned)(cols * (L.T[2] / zp));
#if PINC_MG_SWEEP4C
	hipLaunchKernelGGL((k_gs_sweep4c<32, 8, 256>), dim3(nb), dim3(256), 0, (hipStream_t)stream, phiIn, phiOut, rho, L,
	                   zp);
#else
	hipLaunchKernelGGL((k_gs_sweep4<32, 8, 256>), dim3(nb), dim3(256), 0, (hipStream_t)stream, phiIn, phiOut, rho, L,
	                   zp);
#endif
	return check_launch("gs_sweep2x");
}

extern "C" int pinc_hip_mg_solve_small(double *phi, const double *rho, double *res, int nLevels,
                                       const pinc_lvl_t *levels, int nPre, int nPost, int nCoarse, int maxCycles,
                                       double tol, const double *coarseBasis, double *out, void *stream) {
	if (nLevels < 2 || nLevels > 13) return set_error(hipErrorInvalidValue, "mg_solve_small: 2..13 levels");
	if (levels[0].nd != 2) return set_error(hipErrorInvalidValue, "mg_solve_small: 2-D levels");
	const int T0 = levels[0].T[0], T1 = levels[0].T[1];
	int lg = 0;
	while ((1 << lg) < T0) lg++;
	if ((1 << lg) != T0 || T0 < 2 || T0 > 1024 || T1 % 2 || (long)T0 * T1 > kSmallMax || ((long)T0 * T1) % 2048)
		return set_error(hipErrorInvalidValue,
		                 "mg_solve_small: level 0 not T0 = 2^k <= 1024, T1 even, T0 T1 <= 16384 in 2048s");
	if (maxCycles < 1 || maxCycles > 1000000) return set_error(hipErrorInvalidValue, "mg_solve_small: maxCycles");
	SmallArgs a;
	long tot = 0;
	a.c.nLevels = nLevels - 1;
	for (int l = 1; l < nLevels; l++) {
		if (levels[l].nd != 2) return set_error(hipErrorInvalidValue, "mg_solve_small: mixed dimensions");
		long n = 1;
		for (int d = 0; d < 3; d++) {
			if (d < 2 && 2 * levels[l].T[d] != levels[l - 1].T[d])
				return set_error(hipErrorInvalidValue, "mg_solve_small: levels must halve");
			a.c.T[l - 1][d] = levels[l].T[d];
			n *= levels[l].T[d];
		}
		tot += 3 * n;
	}
	if (tot > kCoarseLds) return set_error(hipErrorInvalidValue, "mg_solve_small: levels exceed the LDS budget");
	a.c.nPre = nPre;
	a.c.nPost = nPost;
	a.c.nCoarse = nCoarse;
	a.c.hw3d = 0;
	a.c.gs3d = 0;
	a.T0[0] = T0;
	a.T0[1] = T1;
	a.lgH = lg - 1;
	a.nPre = nPre;
	a.nPost = nPost;
	a.maxCycles = maxCycles;
	a.tol = tol;
	if (coarseBasis) {
		const int n = levels[1].T[0];
		if (levels[1].T[1] != n || n % 16 || n > 64 || 3 * n * (n + 1) + n > kCoarseLds)
			return set_error(hipErrorInvalidValue, "mg_solve_small: the spectral level 1 must be square, n = 16, 32, 48, 64");
	}
	// one instance per slot count (compile-time: unrolled slot loops with
	// the thread's rho in fixed registers)
	const int P = (T0 * T1) >> 10;
	if (P != 2 && P != 4 && P != 8 && P != 16)
		return set_error(hipErrorInvalidValue, "mg_solve_small: level 0 of 2048, 4096, 8192 or 16384 points");
	auto kern = coarseBasis ? (P == 2 ? k_mg_solve_small2<true, 2>
	                           : P == 4 ? k_mg_solve_small2<true, 4>
	                           : P == 8 ? k_mg_solve_small2<true, 8>
	                                    : k_mg_solve_small2<true, 16>)
	                        : (P == 2 ? k_mg_solve_small2<false, 2>
	                           : P == 4 ? k_mg_solve_small2<false, 4>
	                           : P == 8 ? k_mg_solve_small2<false, 8>
	                                    : k_mg_solve_small2<false, 16>);
	hipLaunchKernelGGL(kern, dim3(1), dim3(1024), 0, (hipStream_t)stream, phi, rho, res, a, out, coarseBasis);
	return check_launch("mg_solve_small");
}

extern "C" int pinc_hip_mg_coarse(const double *rho, double *phi, int nLevels, const pinc_lvl_t *levels, int nPre,
                                  int nPost, int nCoarse, int hw3d, int gs3d, void *stream) {
	CoarseArgs a;
	if (nLevels < 1 || nLevels > 12) return set_error(hipErrorInvalidValue, "mg_coarse: 1..12 levels");
	const int nd = levels[0].nd;
	if (nd < 1 || nd > 3) return set_error(hipErrorInvalidValue, "mg_coarse: 1-3 dimensions");
	if (nd != 3 && (hw3d || gs3d)) return set_error(hipErrorInvalidValue, "mg_coarse: 3-D operators on a non-3-D grid");
	long tot = 0;
	a.nLevels = nLevels;
	for (int l = 0; l < nLevels; l++) {
		if (levels[l].nd != nd) return set_error(hipErrorInvalidValue, "mg_coarse: mixed dimensions");
		long n = 1;
		for (int d = 0; d < 3; d++) {
			a.T[l][d] = levels[l].T[d];
			n *= levels[l].T[d];
			if (l > 0 && d < nd && 2 * levels[l].T[d] != levels[l - 1].T[d])
				return set_error(hipErrorInvalidValue, "mg_coarse: levels must halve");
		}
		tot += 3 * n;
	}
	if (tot > kCoarseLds) return set_error(hipErrorInvalidValue, "mg_coarse: levels exceed the LDS budget");
	a.nPre = nPre;
	a.nPost = nPost;
	a.nCoarse = nCoarse;
	a.hw3d = hw3d;
	a.gs3d = gs3d;
	hipStream_t st = (hipStream_t)stream;
	if (nd == 3) hipLaunchKernelGGL(k_mg_coarse<3>, dim3(1), dim3(1024), 0, st, rho, phi, a);
	else if (nd == 2) hipLaunchKernelGGL(k_mg_coarse<2>, dim3(1), dim3(1024), 0, st, rho, phi, a);
	else hipLaunchKernelGGL(k_mg_coarse<1>, dim3(1), dim3(1024), 0, st, rho, phi, a);
	return check_launch("mg_coarse");
}

extern "C" int pinc_hip_residual_slab(double *res, const double *phi, const double *rho, pinc_lvl_t Lx, int zlo,
                                      int zhi, void *stream) {
	if (npts(Lx) >= (1L << 31)) return set_error(hipErrorInvalidValue, "residual_slab: level too large for 32-bit indexing");
	if (Lx.nd != 3 || zlo < 1 || zhi > Lx.T[2] - 1 || zhi <= zlo)
		return set_error(hipErrorInvalidValue, "residual_slab: planes must have both z neighbours in the slab");
	long n = (long)Lx.T[0] * Lx.T[1] * (zhi - zlo);
	hipLaunchKernelGGL(k_residual_slab<false>, dim3(blocks_for(n)), dim3(kThreads), 0, (hipStream_t)stream, res, phi,
	                   rho, Lx, zlo, zhi);
	return check_launch("residual_slab");
}

extern "C" int pinc_hip_residual_sumsq_slab(const double *phi, const double *rho, pinc_lvl_t Lx, int zlo, int zhi,
                                            double *partial, int *nBlocks, void *stream) {
	if (npts(Lx) >= (1L << 31)) return set_error(hipErrorInvalidValue, "residual_sumsq_slab: level too large for 32-bit indexing");
	if (Lx.nd != 3 || zlo < 1 || zhi > Lx.T[2] - 1 || zhi <= zlo)
		return set_error(hipErrorInvalidValue, "residual_sumsq_slab: planes must have both z neighbours in the slab");
	long n = (long)Lx.T[0] * Lx.T[1] * (zhi - zlo);
	unsigned nb = blocks_for(n);
	*nBlocks = (int)nb;
	hipLaunchKernelGGL(k_residual_slab<true>, dim3(nb), dim3(kThreads), 0, (hipStream_t)stream, partial, phi, rho, Lx,
	                   zlo, zhi);
	return check_launch("residual_sumsq_slab");
}

extern "C" int pinc_hip_restrict_slab(const double *fineX, pinc_lvl_t Lx, int zf0, double *coarse, pinc_lvl_t Lc,
                                      int nd3, void *stream) {
	if (npts(Lc) >= (1L << 31)) return set_error(hipErrorInvalidValue, "restrict_slab: level too large for 32-bit indexing");
	if (Lx.nd != 3 || Lc.nd != 3 || 2 * Lc.T[0] != Lx.T[0] || 2 * Lc.T[1] != Lx.T[1] || zf0 < 1 ||
	    zf0 + 2 * Lc.T[2] > Lx.T[2])
		return set_error(hipErrorInvalidValue, "restrict_slab: geometry");
	unsigned nb = blocks_for(npts(Lc));
	hipStream_t st = (hipStream_t)stream;
	if (nd3) hipLaunchKernelGGL(k_restrict_slab<true>, dim3(nb), dim3(kThreads), 0, st, fineX, Lx, zf0, coarse, Lc);
	else hipLaunchKernelGGL(k_restrict_slab<false>, dim3(nb), dim3(kThreads), 0, st, fineX, Lx, zf0, coarse, Lc);
	return check_launch("restrict_slab");
}

extern "C" int pinc_hip_prolong_add_own(double *phiX, pinc_lvl_t Lx, int hz, int nloc, const double *phiCx,
                                        pinc_lvl_t Lcx, void *stream) {
	if (Lx.nd != 3 || Lcx.nd != 3 || 2 * Lcx.T[0] != Lx.T[0] || 2 * Lcx.T[1] != Lx.T[1] || nloc % 2 ||
	    2 * (Lcx.T[2] - 2) != nloc || hz < 0 || hz + nloc > Lx.T[2])
		return set_error(hipErrorInvalidValue, "prolong_add_own: geometry");
	if ((long)Lx.T[0] * Lx.T[1] * nloc >= (1L << 31))
		return set_error(hipErrorInvalidValue, "prolong_add_own: slab too large for 32-bit indexing");
	const long n = (long)Lx.T[0] * Lx.T[1] * nloc;
	hipLaunchKernelGGL(k_prolong_add_own, dim3(blocks_for(n)), dim3(kThreads), 0, (hipStream_t)stream, phiX, Lx, hz,
	                   nloc, phiCx, Lcx);
	return check_launch("prolong_add_own");
}

extern "C" int pinc_hip_prolong_add_slab(double *phiX, pinc_lvl_t Lx, int z0, int Tz, const double *phiC,
                                         pinc_lvl_t Lc, void *stream) {
	if (Lx.nd != 3 || Lc.nd != 3 || 2 * Lc.T[0] != Lx.T[0] || 2 * Lc.T[1] != Lx.T[1] || 2 * Lc.T[2] != Tz)
		return set_error(hipErrorInvalidValue, "prolong_add_slab: geometry");
	hipLaunchKernelGGL(k_prolong_add_slab, dim3(blocks_for(npts(Lx))), dim3(kThreads), 0, (hipStream_t)stream, phiX,
	                   Lx, z0, Tz, phiC, Lc);
	return check_launch("prolong_add_slab");
}
