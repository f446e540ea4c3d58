/*
 * ORACLE TEST INFRASTRUCTURE -- never linked into the product.
 *
 * Binds the firmware's `pow10f` calls (audio_agc.c:260-328, audio_driver.c:914,943)
 * to glibc's own pow10f, which this image's libm still exports as the versioned
 * compatibility symbol pow10f@GLIBC_2.2.5 (it was only dropped from the headers in
 * glibc 2.27).  No replacement implementation is supplied: the symbol resolves to
 * the library function that ships in /lib/x86_64-linux-gnu/libm.so.6.
 */
#ifndef UHSDR_POW10F_GLIBC_H
#define UHSDR_POW10F_GLIBC_H
float pow10f(float x);
__asm__(".symver pow10f,pow10f@GLIBC_2.2.5");
#endif
