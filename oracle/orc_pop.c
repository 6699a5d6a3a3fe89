/*
 * orc_pop.c -- TEST INFRASTRUCTURE (oracle).  Restates src/population.c:
 *   op_alloc          pAlloc          population.c:42-92
 *   op_pos_lattice    pPosLattice     population.c:172-240
 *   op_pos_perturb    pPosPerturb     population.c:242-276
 *   op_vel_zero       pVelZero        population.c:412-428
 *   op_vel_maxwell    pVelMaxwell     population.c:367-392 (own counter RNG:
 *                     GSL's mt19937/ziggurat is absent -> draws unpinned)
 *   op_to_local/glob  pToLocalFrame   population.c:727-763
 *   op_sum_kin        pSumKinEnergy   population.c:700-709
 * Particles also carry a shadow id (lattice index) so tests can match
 * particles across implementations whose storage order may differ.
 */
#include "orc.h"
#include <math.h>

void op_alloc(OPop *p, const OIni *ini, int mpiSize){
	memset(p, 0, sizeof(*p));
	int nSpecies = oini_int(ini, "population:nSpecies");
	int nDims = oini_int(ini, "grid:nDims");
	long *tot = oini_longarr(ini, "population:nAlloc", nSpecies);
	p->nSpecies = nSpecies;
	p->nDims = nDims;
	p->iStart = malloc((nSpecies+1)*sizeof(long));
	p->iStop = malloc(nSpecies*sizeof(long));
	p->iStart[0] = 0;
	for(int s = 1; s <= nSpecies; s++)
		p->iStart[s] = p->iStart[s-1] + (long)ceil((double)tot[s-1]/mpiSize);
	for(int s = 0; s < nSpecies; s++) p->iStop[s] = p->iStart[s];
	long n = p->iStart[nSpecies];
	p->pos = calloc((size_t)nDims*n, sizeof(double));
	p->vel = calloc((size_t)nDims*n, sizeof(double));
	p->id = calloc(n ? n : 1, sizeof(long));
	p->charge = oini_doublearr(ini, "population:charge", nSpecies);
	p->mass = oini_doublearr(ini, "population:mass", nSpecies);
	p->kinEnergy = calloc(nSpecies+1, sizeof(double));
	p->potEnergy = calloc(nSpecies+1, sizeof(double));
	free(tot);
}

void op_free(OPop *p){
	free(p->pos); free(p->vel); free(p->id); free(p->iStart); free(p->iStop);
	free(p->charge); free(p->mass); free(p->kinEnergy); free(p->potEnergy);
}

void op_to_local(OPop *p, const OMpi *mpi){
	int nd = p->nDims;
	for(int s = 0; s < p->nSpecies; s++)
		for(long i = p->iStart[s]; i < p->iStop[s]; i++)
			for(int d = 0; d < nd; d++) p->pos[i*nd+d] -= mpi->offset[d];
}

void op_to_global(OPop *p, const OMpi *mpi){
	int nd = p->nDims;
	for(int s = 0; s < p->nSpecies; s++)
		for(long i = p->iStart[s]; i < p->iStop[s]; i++)
			for(int d = 0; d < nd; d++) p->pos[i*nd+d] += mpi->offset[d];
}

static void global_size(const OIni *ini, int nDims, int *L, long *V){
	int *ts = oini_intarr(ini, "grid:trueSize", nDims);
	int *ns = oini_intarr(ini, "grid:nSubdomains", nDims);
	long v = 1;
	for(int d = 0; d < nDims; d++){ L[d] = ns[d]*ts[d]; v *= L[d]; }
	*V = v;
	free(ts); free(ns);
}

void op_pos_lattice(OPop *p, const OIni *ini, const OMpi *mpi){
	int nd = p->nDims;
	long *nPart = oini_longarr(ini, "population:nParticles", p->nSpecies);
	int L[3]; long V;
	global_size(ini, nd, L, &V);
	for(int s = 0; s < p->nSpecies; s++){
		double l = pow(V/(double)nPart[s], 1.0/nd);
		long iStop = p->iStart[s];
		for(long i = 0; i < nPart[s]; i++){
			double x[3];
			double lin = l*i;
			for(int d = 0; d < nd; d++){
				x[d] = fmod(lin, L[d]);
				lin /= L[d];
			}
			int ok = 0;
			for(int d = 0; d < nd; d++)
				ok += (mpi->subdomain[d] == (int)(mpi->posToSubdomain[d]*x[d]));
			if(ok == nd){
				if(iStop >= p->iStart[s+1]) orc_die("allocated too few particles (species %d)", s);
				for(int d = 0; d < nd; d++) p->pos[iStop*nd+d] = x[d];
				p->id[iStop] = i;
				iStop++;
			}
		}
		p->iStop[s] = iStop;
	}
	op_to_local(p, mpi);
	free(nPart);
}

void op_pos_perturb(OPop *p, const OIni *ini, const OMpi *mpi){
	int nd = p->nDims, ns = p->nSpecies;
	double *amp = oini_doublearr(ini, "population:perturbAmplitude", nd*ns);
	double *mode = oini_doublearr(ini, "population:perturbMode", nd*ns);
	int L[3]; long V;
	global_size(ini, nd, L, &V);
	op_to_global(p, mpi);
	for(int s = 0; s < ns; s++)
		for(long i = p->iStart[s]; i < p->iStop[s]; i++)
			for(int d = 0; d < nd; d++){
				double theta = 2.0*M_PI*mode[s*nd+d]*p->pos[i*nd+d]/L[d];
				p->pos[i*nd+d] += amp[s*nd+d]*cos(theta);
			}
	op_to_local(p, mpi);
	free(amp); free(mode);
}

void op_vel_zero(OPop *p){
	int nd = p->nDims;
	for(int s = 0; s < p->nSpecies; s++)
		for(long i = p->iStart[s]; i < p->iStop[s]; i++)
			for(int d = 0; d < nd; d++) p->vel[i*nd+d] = 0;
}

/* splitmix64 finaliser as a counter-based generator */
static unsigned long long mix64(unsigned long long z){
	z += 0x9E3779B97F4A7C15ULL;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}

double orc_uniform(unsigned long long seed, unsigned long long counter){
	unsigned long long x = mix64(seed ^ mix64(counter));
	return ((double)(x >> 11) + 0.5)*(1.0/9007199254740992.0);
}

double orc_normal(unsigned long long seed, unsigned long long counter){
	double u1 = orc_uniform(seed, 2*counter), u2 = orc_uniform(seed, 2*counter + 1);
	return sqrt(-2.0*log(u1))*cos(2.0*M_PI*u2);
}

void op_vel_maxwell(OPop *p, const OIni *ini, unsigned long long seed){
	int nd = p->nDims, ns = p->nSpecies;
	double *drift = oini_doublearr(ini, "population:drift", ns);
	double *vth = oini_doublearr(ini, "population:thermalVelocity", ns);
	for(int s = 0; s < ns; s++)
		for(long i = p->iStart[s]; i < p->iStop[s]; i++){
			unsigned long long c = ((unsigned long long)s << 40 | (unsigned long long)p->id[i])*3ULL;
			for(int d = 0; d < nd; d++)
				p->vel[i*nd+d] = drift[s] + vth[s]*orc_normal(seed, c + d);
		}
	free(drift); free(vth);
}

void op_sum_kin(OPop *p){
	int ns = p->nSpecies;
	p->kinEnergy[ns] = 0;
	for(int s = 0; s < ns; s++) p->kinEnergy[ns] += p->kinEnergy[s];
}
