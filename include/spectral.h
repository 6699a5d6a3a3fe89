/*
 * spectral.h -- the reference's header name (src/spectral.h), forwarding to this
 * build's operator surface: main.c:10-13 includes it; every spectral symbol that
 * main.c uses is declared in pinc.h (tests/golden/mainc_symbols.json).
 */
#ifndef PINC_FWD_SPECTRAL_H
#define PINC_FWD_SPECTRAL_H
#include "core.h"
#endif
