/*
 * dk_diag.h — diagnostics shipped in libdk_rx.so that are not part of the receive-path ABI (dk_rx.h).
 */
#ifndef DK_DIAG_H
#define DK_DIAG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Streaming read of `bytes` (multiple of 16) of device memory at `buf`; `scratch` = device u32[grid] (zeroed by the
 * caller). Used to measure the achievable HBM read bandwidth on the running box. Async on `stream`.
 * mode 0: grid-stride loads; 1: contiguous 8 KiB per wave step; 2: as 1 with nontemporal loads.
 * Returns 0, EINVAL or EIO. */
int dk_diag_read_probe(const void* buf, uint64_t bytes, uint32_t* scratch, uint32_t grid, int mode, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DK_DIAG_H */
