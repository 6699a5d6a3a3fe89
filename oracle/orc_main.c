/*
 * orc_main.c -- TEST INFRASTRUCTURE (oracle) command line driver.
 *   orc_run <ini> [--literal] [--noperturb] [--maxwell SEED] [--steps N]
 *           [key=value ...]
 * Prints "n KE PE cycles" per step with %.17g, like the survey harness.
 */
#include "orc.h"
#include <time.h>

OWorld *orc_world_new(const char *iniPath, int nOver, const char **over, int literal);

int main(int argc, char **argv){
	if(argc < 2){ fprintf(stderr, "usage: %s ini [opts] [key=val...]\n", argv[0]); return 2; }
	int literal = 0, perturb = 1, maxwell = 0, steps = -1;
	unsigned long long seed = 0;
	const char *over[256]; int nOver = 0;
	for(int i = 2; i < argc; i++){
		if(!strcmp(argv[i], "--literal")) literal = 1;
		else if(!strcmp(argv[i], "--noperturb")) perturb = 0;
		else if(!strcmp(argv[i], "--maxwell")){ maxwell = 1; seed = strtoull(argv[++i], 0, 10); }
		else if(!strcmp(argv[i], "--steps")) steps = atoi(argv[++i]);
		else over[nOver++] = argv[i];
	}
	OWorld *w = orc_world_new(argv[1], nOver, over, literal);
	if(steps < 0) steps = oini_int(w->ini, "time:nTimeSteps");
	struct timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	ow_init(w, perturb, maxwell, seed);
	ow_init_fields(w);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	fprintf(stderr, "init %.3f s, cycles %ld\n", (t1.tv_sec-t0.tv_sec)+1e-9*(t1.tv_nsec-t0.tv_nsec), w->cycles);
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for(int n = 1; n <= steps; n++){
		ow_step(w);
		printf("%d %.17g %.17g %ld\n", n, w->lastKE, w->lastPE, w->cycles);
		fflush(stdout);
	}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	fprintf(stderr, "loop %.3f s\n", (t1.tv_sec-t0.tv_sec)+1e-9*(t1.tv_nsec-t0.tv_nsec));
	ow_free(w);
	return 0;
}
