/*
 * multigrid.h -- the reference's header name (src/multigrid.h), forwarding to this
 * build's operator surface: main.c:10-13 includes it; every multigrid symbol that
 * main.c uses is declared in pinc.h (tests/golden/mainc_symbols.json).
 */
#ifndef PINC_FWD_MULTIGRID_H
#define PINC_FWD_MULTIGRID_H
#include "core.h"
#endif
