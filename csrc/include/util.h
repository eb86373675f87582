/*
 * util.h -- source compatibility with the reference's util.h
 * (/root/reference/util.h:1-8, used only by commented-out code in
 * /root/reference/test.c:158-171): printh() prints a NUL-terminated byte
 * string as hex.  Unlike the reference, bytes are printed unsigned (the
 * reference sign-extends bytes >= 0x80 to "ffffff80"), and the function is
 * static inline so several translation units may include this header.
 */
#ifndef OTC_UTIL_H
#define OTC_UTIL_H

#include <stdio.h>

static inline void printh(const char *buffer)
{
    for (const unsigned char *p = (const unsigned char *)buffer; *p; ++p) printf("%02x", *p);
    printf("\n");
}

#endif
