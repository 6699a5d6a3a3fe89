/*
 * pusher.h -- the reference's header name (src/pusher.h), forwarding to this
 * build's operator surface: main.c:10-13 includes it; every pusher symbol that
 * main.c uses is declared in pinc.h (tests/golden/mainc_symbols.json).
 */
#ifndef PINC_FWD_PUSHER_H
#define PINC_FWD_PUSHER_H
#include "core.h"
#endif
