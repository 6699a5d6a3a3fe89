/*
 * orc_pusher.c -- TEST INFRASTRUCTURE (oracle).  Restates src/pusher.c:
 *   opu_move        puMove (as compiled: pos += vel)   pusher.c:86-119
 *   opu_acc3d1      puAcc3D1 / puAcc3D1KE              pusher.c:147-214
 *                   + puInterp3D1                      pusher.c:1089-1122
 *   opu_accnd1      puAccND1 / puAccND1KE              pusher.c:219-308
 *                   + puInterpND1(Inner)               pusher.c:1124-1162
 *   opu_distr3d1    puDistr3D1                         pusher.c:512-572
 *   opu_distrnd1    puDistrND1(+Inner)                 pusher.c:578-638
 *   opu_accnd0      puAccND0KE + puInterpND0           pusher.c:310-353, 1164-1180
 *   opu_distrnd0    puDistrND0                         pusher.c:640-668
 *   opu_extract3d   puExtractEmigrants3D               pusher.c:782-855
 *   opu_extractnd   puExtractEmigrantsND               pusher.c:862-910
 *   ow_migrate      puMigrate: exchangeNMigrants,      pusher.c:914-1035
 *                   shiftImmigrants, importParticles, exchangeMigrants
 *   neighbour maps  puNeighborToRank/Reciprocal,       pusher.c:1181-1232
 *                   puRankToNeighbor
 *   om_create_neighborhood  gCreateNeighborhood        grid.c:1029-1132
 * The per-species in-place rescaling of E and rho (gMul by q/m, m/q, 1/q, q)
 * is reproduced because it is part of the reference's rounding.
 *
 * Message order: the reference receives migrants with MPI_ANY_SOURCE.  With
 * one rank all messages are self-sends and arrive in send order, i.e. by the
 * sender's neighbour index ne = 0..26, which is tag = reciprocal(ne) = 26..0.
 * The emulation processes tags 26..0 for every rank, exactly reproducing the
 * one-rank order and giving a fixed, documented order for P > 1.
 */
#include "orc.h"
#include <math.h>

void opu_move(OPop *p){
	int nd = p->nDims;
	for(int s = 0; s < p->nSpecies; s++)
		for(long q = p->iStart[s]*nd; q < p->iStop[s]*nd; q++) p->pos[q] += p->vel[q];
}

static inline void interp3d1(double *res, const double *pos, const double *val, const long *sp){
	int j = (int)pos[0], k = (int)pos[1], l = (int)pos[2];
	double x = pos[0]-j, y = pos[1]-k, z = pos[2]-l;
	double xc = 1-x, yc = 1-y, zc = 1-z;
	long p = j*3 + k*sp[2] + l*sp[3];
	long pj = p + 3, pk = p + sp[2], pjk = pk + 3;
	long pl = p + sp[3], pjl = pl + 3, pkl = pl + sp[2], pjkl = pkl + 3;
	for(int v = 0; v < 3; v++)
		res[v] = zc*( yc*(xc*val[p+v] + x*val[pj+v])
		            + y *(xc*val[pk+v] + x*val[pjk+v]) )
		       + z *( yc*(xc*val[pl+v] + x*val[pjl+v])
		            + y *(xc*val[pkl+v] + x*val[pjkl+v]) );
}

void opu_acc3d1(OPop *p, OGrid *E, int ke){
	const long *sp = E->sizeProd;
	for(int s = 0; s < p->nSpecies; s++){
		og_mul(E, p->charge[s]/p->mass[s]);
		if(ke) p->kinEnergy[s] = 0;
		for(long i = p->iStart[s]; i < p->iStop[s]; i++){
			double dv[3];
			double *v = &p->vel[3*i];
			interp3d1(dv, &p->pos[3*i], E->val, sp);
			double vs = 0;
			for(int d = 0; d < 3; d++){
				vs += v[d]*(v[d]+dv[d]);
				v[d] += dv[d];
			}
			if(ke) p->kinEnergy[s] += vs;
		}
		if(ke) p->kinEnergy[s] *= 0.5*p->mass[s];
		og_mul(E, p->mass[s]/p->charge[s]);
	}
}

/* puBoris3D1 / puBoris3D1KE (pusher.c:394-483) as the algorithm they state,
 * with the indexing corrected (fact 7: the reference rotates vel[0..2], the
 * first particle, instead of vel[p..p+2], and memcpy's the wrong source):
 * v- = v + dv/2; v' = v- + v- x T; v+ = v- + v' x S (addCross,
 * pusher.c:1234-1238, same expression order); KE sums v+^2 (pow(v,2) is the
 * correctly rounded square); v = v+ + dv/2.  T and S per species from
 * puGet3DRotationParameters (pusher.c:485-505). */
static void add_cross(const double *a, const double *b, double *res){
	res[0] +=  (a[1]*b[2]-a[2]*b[1]);
	res[1] += -(a[0]*b[2]-a[2]*b[0]);
	res[2] +=  (a[0]*b[1]-a[1]*b[0]);
}

void opu_boris3d1(OPop *p, OGrid *E, const double *T, const double *S, int ke){
	const long *sp = E->sizeProd;
	for(int s = 0; s < p->nSpecies; s++){
		og_mul(E, p->charge[s]/p->mass[s]);
		if(ke) p->kinEnergy[s] = 0;
		for(long i = p->iStart[s]; i < p->iStop[s]; i++){
			double dv[3], vPrime[3];
			double *v = &p->vel[3*i];
			interp3d1(dv, &p->pos[3*i], E->val, sp);
			for(int d = 0; d < 3; d++) v[d] += 0.5*dv[d];
			for(int d = 0; d < 3; d++) vPrime[d] = v[d];
			add_cross(v, &T[3*s], vPrime);
			add_cross(vPrime, &S[3*s], v);
			double vs = 0;
			for(int d = 0; d < 3; d++) vs += v[d]*v[d];
			if(ke) p->kinEnergy[s] += vs;
			for(int d = 0; d < 3; d++) v[d] += 0.5*dv[d];
		}
		if(ke) p->kinEnergy[s] *= 0.5*p->mass[s];
		og_mul(E, p->mass[s]/p->charge[s]);
	}
}

void opu_rotation_params(int nSpecies, const double *BExt, const double *charge, const double *mass, double *T,
                         double *S){
	for(int s = 0; s < nSpecies; s++){
		double factor = 0.5*charge[s]/mass[s];
		double denom = 1;
		for(int q = 0; q < 3; q++){
			T[3*s+q] = factor*BExt[q];
			denom += T[3*s+q]*T[3*s+q];
		}
		double mul = 2.0/denom;
		for(int q = 0; q < 3; q++) S[3*s+q] = mul*T[3*s+q];
	}
}

/* recursion from the highest dimension down to x; factor carries the product
 * of the weights of the outer dimensions (pusher.c:1147-1162). */
static void interpnd_inner(double *res, const double *val, long p, const long *mul, long lastMul,
                           int nd, const double *dec, const double *comp, double factor){
	if(*mul == lastMul){
		for(int d = 0; d < nd; d++){
			res[d] += *comp*factor*val[p+d];
			res[d] += *dec*factor*val[p+d+*mul];
		}
	} else {
		interpnd_inner(res, val, p, mul-1, lastMul, nd, dec-1, comp-1, *comp*factor);
		interpnd_inner(res, val, p+*mul, mul-1, lastMul, nd, dec-1, comp-1, *dec*factor);
	}
}

void opu_accnd1(OPop *p, OGrid *E, int ke){
	int nd = p->nDims;
	const long *sp = E->sizeProd;
	for(int s = 0; s < p->nSpecies; s++){
		og_mul(E, p->charge[s]/p->mass[s]);
		if(ke) p->kinEnergy[s] = 0;
		for(long i = p->iStart[s]; i < p->iStop[s]; i++){
			double dv[3], dec[3], comp[3];
			const double *x = &p->pos[nd*i];
			double *v = &p->vel[nd*i];
			long q = 0;
			for(int d = 0; d < nd; d++){
				int in = (int)x[d];
				dec[d] = x[d] - in;
				comp[d] = 1 - dec[d];
				q += sp[d+1]*in;
				dv[d] = 0;
			}
			interpnd_inner(dv, E->val, q, &sp[nd], sp[1], nd, &dec[nd-1], &comp[nd-1], 1);
			double vs = 0;
			for(int d = 0; d < nd; d++){
				vs += v[d]*(v[d]+dv[d]);
				v[d] += dv[d];
			}
			if(ke) p->kinEnergy[s] += vs;
		}
		if(ke) p->kinEnergy[s] *= 0.5*p->mass[s];
		og_mul(E, p->mass[s]/p->charge[s]);
	}
}

void opu_distr3d1(const OPop *p, OGrid *rho){
	og_zero(rho);
	double *val = rho->val;
	const long *sp = rho->sizeProd;
	for(int s = 0; s < p->nSpecies; s++){
		og_mul(rho, 1.0/p->charge[s]);
		for(long i = p->iStart[s]; i < p->iStop[s]; i++){
			const double *pos = &p->pos[3*i];
			int j = (int)pos[0], k = (int)pos[1], l = (int)pos[2];
			double x = pos[0]-j, y = pos[1]-k, z = pos[2]-l;
			double xc = 1-x, yc = 1-y, zc = 1-z;
			long q = j + k*sp[2] + l*sp[3];
			long qk = q + sp[2], ql = q + sp[3], qkl = ql + sp[2];
			val[q]      += xc*yc*zc;
			val[q+1]    += x *yc*zc;
			val[qk]     += xc*y *zc;
			val[qk+1]   += x *y *zc;
			val[ql]     += xc*yc*z ;
			val[ql+1]   += x *yc*z ;
			val[qkl]    += xc*y *z ;
			val[qkl+1]  += x *y *z ;
		}
		og_mul(rho, p->charge[s]);
	}
}

static void distrnd_inner(double *val, long p, const long *mul, long lastMul,
                          const double *dec, const double *comp, double factor){
	if(*mul == lastMul){
		val[p] += *comp*factor;
		val[p+*mul] += *dec*factor;
	} else {
		distrnd_inner(val, p, mul-1, lastMul, dec-1, comp-1, *comp*factor);
		distrnd_inner(val, p+*mul, mul-1, lastMul, dec-1, comp-1, *dec*factor);
	}
}

void opu_distrnd1(const OPop *p, OGrid *rho){
	og_zero(rho);
	int nd = p->nDims;
	const long *sp = rho->sizeProd;
	for(int s = 0; s < p->nSpecies; s++){
		og_mul(rho, 1.0/p->charge[s]);
		for(long i = p->iStart[s]; i < p->iStop[s]; i++){
			const double *pos = &p->pos[nd*i];
			double dec[3], comp[3];
			long q = 0;
			for(int d = 0; d < nd; d++){
				int in = (int)pos[d];
				dec[d] = pos[d] - in;
				comp[d] = 1 - dec[d];
				q += in*sp[d+1];
			}
			distrnd_inner(rho->val, q, &sp[nd], sp[1], &dec[nd-1], &comp[nd-1], 1);
		}
		og_mul(rho, p->charge[s]);
	}
}

/* order 0 (nearest grid point): puAccND0KE (pusher.c:310-353) with
 * puInterpND0 (pusher.c:1164-1180), and puDistrND0 (pusher.c:640-668); the
 * node is (int)(x + 0.5) per dimension */
void opu_accnd0(OPop *p, OGrid *E, int ke){
	int nd = p->nDims;
	const long *sp = E->sizeProd;
	for(int s = 0; s < p->nSpecies; s++){
		og_mul(E, p->charge[s]/p->mass[s]);
		if(ke) p->kinEnergy[s] = 0;
		for(long i = p->iStart[s]; i < p->iStop[s]; i++){
			const double *x = &p->pos[nd*i];
			double *v = &p->vel[nd*i];
			long q = 0;
			for(int d = 0; d < nd; d++) q += sp[d+1]*(int)(x[d]+0.5);
			double vs = 0;
			for(int d = 0; d < nd; d++){
				double dv = E->val[q+d];
				vs += v[d]*(v[d]+dv);
				v[d] += dv;
			}
			if(ke) p->kinEnergy[s] += vs;
		}
		if(ke) p->kinEnergy[s] *= 0.5*p->mass[s];
		og_mul(E, p->mass[s]/p->charge[s]);
	}
}

void opu_distrnd0(const OPop *p, OGrid *rho){
	og_zero(rho);
	int nd = p->nDims;
	const long *sp = rho->sizeProd;
	for(int s = 0; s < p->nSpecies; s++){
		og_mul(rho, 1.0/p->charge[s]);
		for(long i = p->iStart[s]; i < p->iStop[s]; i++){
			const double *pos = &p->pos[nd*i];
			long q = 0;
			for(int d = 0; d < nd; d++) q += (int)(pos[d]+0.5)*sp[d+1];
			rho->val[q]++;
		}
		og_mul(rho, p->charge[s]);
	}
}

/* ------------------------------------------------------- neighbourhood -- */
static int ipow3(int d){ int r = 1; while(d--) r *= 3; return r; }

void om_create_neighborhood(OMpi *m, const OIni *ini, const OGrid *g){
	int nd = m->nDims, ns = m->nSpecies;
	int nN = ipow3(nd);
	int center = 0;
	for(int i = 0; i < nd; i++) center += ipow3(i);
	int nTest = oini_nelem(ini, "grid:nEmigrantsAlloc");
	if(nTest != nN && nTest != 1 && nTest != nd)
		orc_die("grid:nEmigrantsAlloc must have 1, nDims or 3^nDims elements");
	long *tmp = oini_longarr(ini, "grid:nEmigrantsAlloc", nTest);
	m->nEmigrantsAlloc = calloc(nN, sizeof(long));
	for(int ne = 0; ne < nN; ne++){
		if(ne == center) continue;
		if(nTest == 1) m->nEmigrantsAlloc[ne] = tmp[0];
		else if(nTest == nN) m->nEmigrantsAlloc[ne] = tmp[ne];
		else {
			/* element index = dimensionality of the shared interface */
			int t = ne, dims = nd;
			for(int d = nd-1; d >= 0; d--){
				int pw = ipow3(d);
				if(t/pw != 1) dims--;
				t %= pw;
			}
			m->nEmigrantsAlloc[ne] = tmp[dims];
		}
	}
	free(tmp);
	double *thr = oini_doublearr(ini, "grid:thresholds", 2*nd);
	for(int i = 0; i < nd; i++) m->thresholds[i] = thr[i];
	for(int i = nd; i < 2*nd; i++) m->thresholds[i] = (g->size[i%nd+1]-1) - thr[i];
	free(thr);
	m->nNeighbors = nN;
	m->center = center;
	m->nEmigrants = calloc(nN*ns, sizeof(long));
	m->nImmigrants = calloc(nN*ns, sizeof(long));
	m->emigrants = calloc(nN, sizeof(double*));
	m->emigrantIds = calloc(nN, sizeof(long*));
	for(int ne = 0; ne < nN; ne++){
		if(ne == center) continue;
		m->emigrants[ne] = malloc((2*nd*m->nEmigrantsAlloc[ne] + 1)*sizeof(double));
		m->emigrantIds[ne] = malloc((m->nEmigrantsAlloc[ne] + 1)*sizeof(long));
	}
}

int opu_neighbor_to_reciprocal(int neighbor, int nDims){
	int r = 0;
	for(int d = 0; d < nDims; d++){
		r += (2 - (neighbor % 3))*ipow3(d);
		neighbor /= 3;
	}
	return r;
}

int opu_neighbor_to_rank(const OMpi *m, int neighbor){
	int rank = 0;
	for(int d = 0; d < m->nDims; d++){
		int n = (neighbor % 3) - 1;
		neighbor /= 3;
		n = (m->subdomain[d] + n + m->nSubdomains[d]) % m->nSubdomains[d];
		rank += n*m->nSubdomainsProd[d];
	}
	return rank;
}

int opu_rank_to_neighbor(const OMpi *m, int rank){
	int neighbor = 0;
	for(int d = 0; d < m->nDims; d++){
		int n = rank % m->nSubdomains[d];
		n = (n - m->subdomain[d] + 1 + m->nSubdomains[d]) % m->nSubdomains[d];
		rank /= m->nSubdomains[d];
		neighbor += n*ipow3(d);
	}
	return neighbor;
}

/* ---------------------------------------------------------- extraction -- */
/* Emigrant found at slot i of species s: copy it out, back-fill from the last
 * live particle, shrink, and re-test the same slot (pusher.c:827-851). */
static void emigrate(OPop *p, OMpi *m, int s, long i, int ne, long *last){
	int nd = p->nDims;
	long cnt = 0;
	for(int t = 0; t < p->nSpecies; t++) cnt += m->nEmigrants[ne*p->nSpecies + t];
	if(cnt >= m->nEmigrantsAlloc[ne]) orc_die("emigrant buffer %d overflow", ne);
	double *buf = m->emigrants[ne] + 2*nd*cnt;
	for(int d = 0; d < nd; d++) buf[d] = p->pos[nd*i+d];
	for(int d = 0; d < nd; d++) buf[nd+d] = p->vel[nd*i+d];
	m->emigrantIds[ne][cnt] = p->id[i];
	m->nEmigrants[ne*p->nSpecies + s]++;
	long j = *last - 1;
	for(int d = 0; d < nd; d++){
		p->pos[nd*i+d] = p->pos[nd*j+d];
		p->vel[nd*i+d] = p->vel[nd*j+d];
	}
	p->id[i] = p->id[j];
	*last = j;
	p->iStop[s]--;
}

void opu_extract3d(OPop *p, OMpi *m){
	memset(m->nEmigrants, 0, m->nNeighbors*p->nSpecies*sizeof(long));
	const double *t = m->thresholds;
	for(int s = 0; s < p->nSpecies; s++){
		long last = p->iStop[s];
		for(long i = p->iStart[s]; i < last; i++){
			double x = p->pos[3*i], y = p->pos[3*i+1], z = p->pos[3*i+2];
			int nx = -(x < t[0]) + (x >= t[3]);
			int ny = -(y < t[1]) + (y >= t[4]);
			int nz = -(z < t[2]) + (z >= t[5]);
			int ne = 13 + nx + 3*ny + 9*nz;
			if(ne != 13){
				emigrate(p, m, s, i, ne, &last);
				i--;
			}
		}
	}
}

void opu_extractnd(OPop *p, OMpi *m){
	int nd = p->nDims;
	memset(m->nEmigrants, 0, m->nNeighbors*p->nSpecies*sizeof(long));
	const double *t = m->thresholds;
	for(int s = 0; s < p->nSpecies; s++){
		long last = p->iStop[s];
		for(long i = p->iStart[s]; i < last; i++){
			int ne = 0;
			for(int d = nd-1; d >= 0; d--){
				double x = p->pos[nd*i+d];
				ne *= 3;
				ne += 1 - (x < t[d]) + (x >= t[nd+d]);
			}
			if(ne != m->center){
				emigrate(p, m, s, i, ne, &last);
				i--;
			}
		}
	}
}

/* ----------------------------------------------------------- migration -- */
void ow_migrate(OWorld *w){
	int ns = w->nSpecies, nd = w->nDims;
	/* exchangeNMigrants: counts sent in direction ne arrive tagged with
	 * reciprocal(ne) at the neighbour in direction ne. */
	for(int r = 0; r < w->P; r++){
		OMpi *m = &w->r[r].mpi;
		for(int ne = 0; ne < m->nNeighbors; ne++){
			if(ne == m->center) continue;
			int dst = opu_neighbor_to_rank(m, ne);
			int tag = opu_neighbor_to_reciprocal(ne, nd);
			memcpy(&w->r[dst].mpi.nImmigrants[tag*ns], &m->nEmigrants[ne*ns], ns*sizeof(long));
		}
	}
	/* exchangeMigrants: receiver r processes tag t = 26..0; the message with
	 * tag t comes from its neighbour in direction t, which sent it in
	 * direction reciprocal(t). */
	for(int r = 0; r < w->P; r++){
		ORank *R = &w->r[r];
		OMpi *m = &R->mpi;
		OPop *p = &R->pop;
		for(int t = m->nNeighbors-1; t >= 0; t--){
			if(t == m->center) continue;
			int src = opu_neighbor_to_rank(m, t);
			int sne = opu_neighbor_to_reciprocal(t, nd);
			const double *buf = w->r[src].mpi.emigrants[sne];
			const long *ids = w->r[src].mpi.emigrantIds[sne];
			const long *cnt = &m->nImmigrants[t*ns];
			long k = 0;
			for(int s = 0; s < ns; s++){
				if(p->iStop[s] + cnt[s] > p->iStart[s+1]) orc_die("population overflow on import");
				for(long i = 0; i < cnt[s]; i++, k++){
					long dstI = p->iStop[s]++;
					int tt = t;
					for(int d = 0; d < nd; d++){
						int n = tt % 3 - 1;
						tt /= 3;
						double shift = n*R->rho.trueSize[d+1];
						p->pos[nd*dstI+d] = buf[2*nd*k+d] + shift;
					}
					for(int d = 0; d < nd; d++) p->vel[nd*dstI+d] = buf[2*nd*k+nd+d];
					p->id[dstI] = ids[k];
				}
			}
		}
	}
}
