/* cpu_crc32.h -- the library's own host CRC-32 engines (cpu_crc32.c). Raw
 * reflected register in and out (no init / xorout), as val_crc32_update_state. */
#ifndef VCRC_CPU_CRC32_H
#define VCRC_CPU_CRC32_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { VCRC_CPU_BEST = 0, VCRC_CPU_SLICE16 = 1, VCRC_CPU_CLMUL = 2, VCRC_CPU_VPCLMUL = 3 };

uint32_t vcrc_cpu_update(uint32_t state, const void *data, size_t len);
/* engine: VCRC_CPU_*; an engine the CPU lacks falls back to the next simpler one */
uint32_t vcrc_cpu_update_with(int engine, uint32_t state, const void *data, size_t len);
/* the engine vcrc_cpu_update uses on this CPU */
int vcrc_cpu_engine(void);

#ifdef __cplusplus
}
#endif
#endif
