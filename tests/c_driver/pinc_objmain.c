/*
 * pinc_objmain.c -- a C caller of libpinc.so that drives the immersed-object
 * loop through the reference's own API, in the order of src/main.c:84-274
 * (TEST DRIVER, ADVICE r02 "high"): oAlloc, oComputeCapacitanceMatrix,
 * oCollectObjectCharge into a caller-owned rhoObj grid, gAddTo(rho, rhoObj),
 * solve, oApplyCapacitanceMatrix, solve.  Unlike regular() it never attaches
 * the object to the population before the first collection, which is the
 * path a maintainer's main.c takes.  The second FROMHALO fold of main.c:232
 * is left out (the single-add loop), so the run is
 * comparable with regular()'s object loop.
 *
 *   pinc_objmain <file.ini> [section:key=value ...]
 *
 * Prints "STATUS: KE <ke> PE <pe>" and "STATUS: N <particles>" per step.
 */
#include <stdio.h>
#include <stdlib.h>
#include <sys/select.h>   /* before pinc.h, which defines the select() macro */
#include "pinc.h"

int main(int argc, char *argv[]) {
	dictionary *ini = iniOpen(argc, argv);
	void (*acc)(Population *, Grid *) =
	    (void (*)(Population *, Grid *))select(ini, "methods:acc", puAcc3D1KE_set, puAccND1KE_set);
	void (*distr)(const Population *, Grid *) =
	    (void (*)(const Population *, Grid *))select(ini, "methods:distr", puDistr3D1_set, puDistrND1_set);
	void (*extractEmigrants)(Population *, MpiInfo *) = (void (*)(Population *, MpiInfo *))select(
	    ini, "methods:migrate", puExtractEmigrants3D_set, puExtractEmigrantsND_set);
	void (*solverInterface)() = select(ini, "methods:poisson", mgSolver_set);
	void (*solve)() = NULL;
	void *(*solverAlloc)() = NULL;
	void (*solverFree)() = NULL;
	((void (*)(void (**)(), void *(**)(), void (**)()))solverInterface)(&solve, &solverAlloc, &solverFree);

	Units *units = uAlloc(ini);
	uNormalize(ini, units);
	MpiInfo *mpiInfo = gAllocMpi(ini);
	Population *pop = pAlloc(ini);
	Grid *E = gAlloc(ini, VECTOR);
	Grid *rho = gAlloc(ini, SCALAR);
	Grid *rhoObj = gAlloc(ini, SCALAR);
	Grid *phi = gAlloc(ini, SCALAR);
	void *solver = ((void *(*)(const dictionary *, Grid *, Grid *))solverAlloc)(ini, rho, phi);
	void (*solveFn)(void *, Grid *, Grid *, const MpiInfo *) = (void (*)(void *, Grid *, Grid *, const MpiInfo *))solve;
	Object *obj = oAlloc(ini);
	gCreateNeighborhood(ini, mpiInfo, rho);
	gSetBndSlices(phi, mpiInfo);

	/* main.c:141-166 (with pPosPerturb re-enabled, as the harness) */
	oComputeCapacitanceMatrix(obj, ini, mpiInfo);
	pPosLattice(ini, pop, mpiInfo);
	pVelZero(pop);
	pPosPerturb(ini, pop, mpiInfo);
	pSyncToDevice(pop);
	extractEmigrants(pop, mpiInfo);
	puMigrate(pop, mpiInfo, rho);
	gZero(rhoObj);
	oCollectObjectCharge(pop, rhoObj, obj, mpiInfo);
	gZero(rhoObj);

	/* main.c:168-186 */
	distr(pop, rho);
	gHaloOp((funPtr)addSlice, rho, mpiInfo, FROMHALO);
	solveFn(solver, rho, phi, mpiInfo);
	gFinDiff1st(phi, E);
	gHaloOp((funPtr)setSlice, E, mpiInfo, TOHALO);
	gMul(E, -1.);
	gMul(E, 0.5);
	acc(pop, E);
	gMul(E, 2.0);

	/* main.c:197-274 */
	int nTimeSteps = iniGetInt(ini, "time:nTimeSteps");
	for (int n = 1; n <= nTimeSteps; n++) {
		puMove(pop, obj);
		extractEmigrants(pop, mpiInfo);
		puMigrate(pop, mpiInfo, rho);
		oCollectObjectCharge(pop, rhoObj, obj, mpiInfo);
		distr(pop, rho);
		gHaloOp((funPtr)addSlice, rho, mpiInfo, FROMHALO);
		gAddTo(rho, rhoObj);
		solveFn(solver, rho, phi, mpiInfo);
		oApplyCapacitanceMatrix(rho, phi, obj, mpiInfo);
		solveFn(solver, rho, phi, mpiInfo);
		gHaloOp((funPtr)setSlice, phi, mpiInfo, TOHALO);
		gFinDiff1st(phi, E);
		gHaloOp((funPtr)setSlice, E, mpiInfo, TOHALO);
		gMul(E, -1.);
		acc(pop, E);
		pSumKinEnergy(pop);
		gPotEnergy(rho, phi, pop);
		long np = 0;
		for (int s = 0; s < pop->nSpecies; s++) np += pop->iStop[s] - pop->iStart[s];
		msg(STATUS, "KE %.17g PE %.17g", pop->kinEnergy[pop->nSpecies], pop->potEnergy[pop->nSpecies]);
		msg(STATUS, "N %ld", np);
	}

	((void (*)(void *))solverFree)(solver);
	oFree(obj);
	gFree(rho);
	gFree(rhoObj);
	gFree(phi);
	gFree(E);
	pFree(pop);
	gFreeMpi(mpiInfo);
	uFree(units);
	iniClose(ini);
	msg(STATUS, "PINC completed successfully!");
	return 0;
}
