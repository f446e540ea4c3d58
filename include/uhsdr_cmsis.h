/*
 * CMSIS-DSP signature shims executed on the MI355X (libuhsdr_cmsis.so).
 *
 * The firmware's DSP path calls these CMSIS-DSP V1.4.5 f32 functions on caller-owned instance
 * structs, host buffers and state arrays.  This library exports the same
 * symbol names with the same instance layouts and argument meaning
 * (basesw/ovi40/Drivers/CMSIS/Include/arm_math.h), so reference code links against it
 * unchanged; each call copies its block and the instance's state to the device, runs a HIP
 * kernel, and writes the outputs and the updated state back exactly where CMSIS leaves them.
 * Results are bit-identical to the reference's CMSIS build (tests/test_gpu_cmsis.py).
 *
 * These are single-instance, host-pointer calls: each costs a few microseconds of launch and
 * copy latency.  They exist for drop-in linking; throughput comes from the batched ABI in
 * uhsdr.h.  Link this library instead of CMSIS-DSP's f32 filtering / transform objects, not
 * beside them.
 *
 * Errors: CMSIS processing functions return void.  A device failure (or an fftLen other than
 * 16, 32, ..., 4096 in arm_cfft_f32) leaves pDst untouched and is reported by
 * uhsdr_cmsis_last_status() / uhsdr_last_error() (libuhsdr_amd.so).
 */
#ifndef UHSDR_CMSIS_H
#define UHSDR_CMSIS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef float float32_t;

/* arm_math.h:375-382 */
typedef enum
{
    ARM_MATH_SUCCESS = 0,
    ARM_MATH_ARGUMENT_ERROR = -1,
    ARM_MATH_LENGTH_ERROR = -2,
    ARM_MATH_SIZE_MISMATCH = -3,
    ARM_MATH_NANINF = -4,
    ARM_MATH_SINGULAR = -5,
    ARM_MATH_TEST_FAILURE = -6
} arm_status;

/* arm_math.h:1059-1064 -- replaces arm_fir_f32 (FilteringFunctions/arm_fir_f32.c) */
typedef struct
{
    uint16_t numTaps;
    float32_t* pState;     /* numTaps + blockSize - 1 */
    float32_t* pCoeffs;    /* numTaps, time-reversed */
} arm_fir_instance_f32;

void arm_fir_init_f32(arm_fir_instance_f32* S, uint16_t numTaps, float32_t* pCoeffs, float32_t* pState,
                      uint32_t blockSize);
void arm_fir_f32(const arm_fir_instance_f32* S, float32_t* pSrc, float32_t* pDst, uint32_t blockSize);

/* arm_math.h:3291-3297 -- replaces arm_fir_decimate_f32 */
typedef struct
{
    uint8_t M;
    uint16_t numTaps;
    float32_t* pCoeffs;
    float32_t* pState;     /* numTaps + blockSize - 1 */
} arm_fir_decimate_instance_f32;

arm_status arm_fir_decimate_init_f32(arm_fir_decimate_instance_f32* S, uint16_t numTaps, uint8_t M,
                                     float32_t* pCoeffs, float32_t* pState, uint32_t blockSize);
void arm_fir_decimate_f32(const arm_fir_decimate_instance_f32* S, float32_t* pSrc, float32_t* pDst,
                          uint32_t blockSize);

/* arm_math.h:3454-3460 -- replaces arm_fir_interpolate_f32 */
typedef struct
{
    uint8_t L;
    uint16_t phaseLength;
    float32_t* pCoeffs;    /* L * phaseLength */
    float32_t* pState;     /* phaseLength + blockSize - 1 */
} arm_fir_interpolate_instance_f32;

arm_status arm_fir_interpolate_init_f32(arm_fir_interpolate_instance_f32* S, uint8_t L, uint16_t numTaps,
                                        float32_t* pCoeffs, float32_t* pState, uint32_t blockSize);
void arm_fir_interpolate_f32(const arm_fir_interpolate_instance_f32* S, float32_t* pSrc, float32_t* pDst,
                             uint32_t blockSize);

/* arm_math.h:3860-3866 -- replaces arm_iir_lattice_f32 */
typedef struct
{
    uint16_t numStages;
    float32_t* pState;     /* numStages + blockSize */
    float32_t* pkCoeffs;   /* numStages */
    float32_t* pvCoeffs;   /* numStages + 1 */
} arm_iir_lattice_instance_f32;

void arm_iir_lattice_init_f32(arm_iir_lattice_instance_f32* S, uint16_t numStages, float32_t* pkCoeffs,
                              float32_t* pvCoeffs, float32_t* pState, uint32_t blockSize);
void arm_iir_lattice_f32(const arm_iir_lattice_instance_f32* S, float32_t* pSrc, float32_t* pDst,
                         uint32_t blockSize);

/* arm_math.h:1242-1247 -- replaces arm_biquad_cascade_df1_f32 */
typedef struct
{
    uint32_t numStages;
    float32_t* pState;     /* 4 * numStages: x[n-1], x[n-2], y[n-1], y[n-2] per stage */
    float32_t* pCoeffs;    /* 5 * numStages: b0, b1, b2, a1, a2 per stage */
} arm_biquad_casd_df1_inst_f32;

void arm_biquad_cascade_df1_init_f32(arm_biquad_casd_df1_inst_f32* S, uint8_t numStages, float32_t* pCoeffs,
                                     float32_t* pState);
void arm_biquad_cascade_df1_f32(const arm_biquad_casd_df1_inst_f32* S, float32_t* pSrc, float32_t* pDst,
                                uint32_t blockSize);

/* arm_math.h:2141-2147 -- replaces arm_cfft_f32 (TransformFunctions/arm_cfft_f32.c:574-628) for
   every length CMSIS dispatches, 16 ... 4096.  256 / 512 / 1024 (the firmware's spectrum display)
   run the one-wave transform of the spectrum kernels on the library's own copies of the CMSIS
   tables; the other lengths run on the instance's pTwiddle / pBitRevTable (arm_const_structs.c),
   which must be set as CMSIS sets them. */
typedef struct
{
    uint16_t fftLen;
    const float32_t* pTwiddle;
    const uint16_t* pBitRevTable;
    uint16_t bitRevLength;
} arm_cfft_instance_f32;

void arm_cfft_f32(const arm_cfft_instance_f32* S, float32_t* p1, uint8_t ifftFlag, uint8_t bitReverseFlag);

/* arm_math.h:6312 -- replaces arm_cmplx_mag_f32 (ComplexMathFunctions/arm_cmplx_mag_f32.c) */
void arm_cmplx_mag_f32(float32_t* pSrc, float32_t* pDst, uint32_t numSamples);

/* arm_math.h:4119-4127 -- replaces arm_lms_norm_f32 (FilteringFunctions/arm_lms_norm_f32.c), the
   firmware's LMS auto notch (AudioDriver_NotchFilter, audio_driver.c:1755; in-place: pErr may be
   pSrc).  The coefficients in pCoeffs adapt in place; energy and x0 carry in the instance. */
typedef struct
{
    uint16_t numTaps;
    float32_t* pState;     /* numTaps + blockSize - 1 */
    float32_t* pCoeffs;    /* numTaps */
    float32_t mu;
    float32_t energy;
    float32_t x0;
} arm_lms_norm_instance_f32;

void arm_lms_norm_init_f32(arm_lms_norm_instance_f32* S, uint16_t numTaps, float32_t* pCoeffs, float32_t* pState,
                           float32_t mu, uint32_t blockSize);
void arm_lms_norm_f32(arm_lms_norm_instance_f32* S, float32_t* pSrc, float32_t* pRef, float32_t* pOut,
                      float32_t* pErr, uint32_t blockSize);

/* status of the last shim call on this thread: 0 ok, UHSDR_* error code (uhsdr.h) otherwise */
int32_t uhsdr_cmsis_last_status(void);

#ifdef __cplusplus
}
#endif

#endif /* UHSDR_CMSIS_H */
