/*
 * pinc_main.c -- a C caller of libpinc.so in the shape of the reference's
 * src/main.c:19-48 (TEST DRIVER): parse the ini named on
 * the command line plus key=value overrides (iniOpen, io.c:254-311), pick the
 * run mode through select() (main.c:32), run it, close the ini.  No Python
 * and no torch in the process: this is how a maintainer's main.c links the
 * MI355X operator surface.
 *
 *   pinc_main <file.ini> [section:key=value ...]
 */
#include <stdio.h>
#include <stdlib.h>
#include <sys/select.h>   /* before pinc.h, which defines the select() macro */
#include "pinc.h"

int main(int argc, char *argv[]) {
	dictionary *ini = iniOpen(argc, argv);
	msg(STATUS, "PINC (MI355X hot path) started.");
	void (*run)(dictionary *) = (void (*)(dictionary *))select(ini, "methods:mode", regular_set);
	run(ini);
	iniClose(ini);
	msg(STATUS, "PINC completed successfully!");
	return 0;
}
