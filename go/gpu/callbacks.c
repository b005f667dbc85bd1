// SPDX-License-Identifier: Apache-2.0
//
// C function pointers for the ledger callbacks exported from block.go. A Go
// file with //export may only declare in its preamble, so the adapters (which
// restore the ABI's const qualifiers) live here.
#include "_cgo_export.h"
#include "ftsamd.h"

static int get_state_tramp(void* u, const char* k, size_t kl, const uint8_t** v, size_t* vl) {
  return goGetState(u, (char*)k, kl, (uint8_t**)v, vl);
}

static int get_states_tramp(void* u, size_t n, const ftz_bytes* keys, ftz_bytes* vals) {
  return goGetStates(u, n, (ftz_bytes*)keys, vals);
}

ftz_get_state_fn ftz_go_get_state_fn(void) { return get_state_tramp; }
ftz_get_states_fn ftz_go_get_states_fn(void) { return get_states_tramp; }
