/* image_png.c -- PNG texture decode and the format dispatch of libpgrt_image.so.
 *
 * Texture::Texture (APP/texture.cpp:5-54) asks FreeImage for the file type by signature
 * (FreeImage_GetFileType, :15), falls back to the file name (:19), loads the file and converts
 * it with FreeImage_ConvertToRawBits(..., topdown = TRUE) (:46): BGR(A) bytes, top row first,
 * rows FreeImage_GetPitch bytes apart (width * bytes-per-pixel rounded up to 4).  PNG is
 * lossless, so libpng (/opt/conda/lib/libpng16 in this image) yields FreeImage's bytes: RGB ->
 * BGR (3 bytes per pixel), RGBA -> BGRA (4); palette and greyscale images are expanded to RGB(A)
 * and 16-bit samples reduced to 8 (FreeImage keeps palettes / 8-bit grey; no reference asset is
 * either -- data/test3.png, test4.png are RGBA).
 */
#define _POSIX_C_SOURCE 200809L
#include <png.h>
#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "pgrt_image.h"

static char g_err[512];

const char* pgrt_png_error(void) { return g_err; }

int pgrt_png_decode(const char* path, int* width, int* height, int* bpp, int* pitch, unsigned char* out,
                    size_t out_size) {
    g_err[0] = 0;
    FILE* f = fopen(path, "rb");
    if (!f) {
        snprintf(g_err, sizeof g_err, "cannot open %s", path);
        return -1;
    }
    png_structp ps = png_create_read_struct(PNG_LIBPNG_VER_STRING, NULL, NULL, NULL);
    png_infop pi = ps ? png_create_info_struct(ps) : NULL;
    png_bytep* volatile rows = NULL; /* freed after a longjmp */
    if (!ps || !pi) {
        snprintf(g_err, sizeof g_err, "%s: libpng initialisation failed", path);
        png_destroy_read_struct(&ps, &pi, NULL);
        fclose(f);
        return -1;
    }
    if (setjmp(png_jmpbuf(ps))) {
        snprintf(g_err, sizeof g_err, "%s: not a readable PNG", path);
        free((void*)rows);
        png_destroy_read_struct(&ps, &pi, NULL);
        fclose(f);
        return -1;
    }
    png_init_io(ps, f);
    png_read_info(ps, pi);
    const int ct = png_get_color_type(ps, pi);
    if (png_get_bit_depth(ps, pi) == 16) png_set_strip_16(ps);
    if (ct == PNG_COLOR_TYPE_PALETTE) png_set_palette_to_rgb(ps);
    if (ct == PNG_COLOR_TYPE_GRAY || ct == PNG_COLOR_TYPE_GRAY_ALPHA) {
        png_set_expand_gray_1_2_4_to_8(ps);
        png_set_gray_to_rgb(ps);
    }
    if (png_get_valid(ps, pi, PNG_INFO_tRNS)) png_set_tRNS_to_alpha(ps);
    png_set_bgr(ps); /* FreeImage's little-endian BGR(A) byte order (FreeImage.h:86-101) */
    png_read_update_info(ps, pi);
    const int w = (int)png_get_image_width(ps, pi), h = (int)png_get_image_height(ps, pi);
    const int ch = (int)png_get_channels(ps, pi);
    const int p = ((w * ch * 8 + 31) / 32) * 4; /* FreeImage_GetPitch */
    *width = w;
    *height = h;
    *bpp = ch;
    *pitch = p;
    if (!out) {
        png_destroy_read_struct(&ps, &pi, NULL);
        fclose(f);
        return 0;
    }
    if (out_size < (size_t)p * (size_t)h) {
        png_destroy_read_struct(&ps, &pi, NULL);
        fclose(f);
        snprintf(g_err, sizeof g_err, "%s: output buffer too small", path);
        return -2;
    }
    memset(out, 0, (size_t)p * (size_t)h);
    rows = (png_bytep*)malloc(sizeof(png_bytep) * (size_t)h);
    if (!rows) {
        png_destroy_read_struct(&ps, &pi, NULL);
        fclose(f);
        snprintf(g_err, sizeof g_err, "%s: out of memory", path);
        return -1;
    }
    for (int y = 0; y < h; ++y) rows[y] = out + (size_t)y * (size_t)p; /* top-down */
    png_read_image(ps, (png_bytepp)rows);
    png_read_end(ps, NULL);
    free((void*)rows);
    png_destroy_read_struct(&ps, &pi, NULL);
    fclose(f);
    return 0;
}

/* FreeImage_GetFileType (by signature) with the file-name fallback, as texture.cpp:15-20 */
static int image_kind(const char* path) {
    unsigned char sig[8] = {0};
    FILE* f = fopen(path, "rb");
    if (f) {
        const size_t n = fread(sig, 1, sizeof sig, f);
        fclose(f);
        if (n >= 3 && sig[0] == 0xFF && sig[1] == 0xD8 && sig[2] == 0xFF) return 1;
        if (n == 8 && png_sig_cmp(sig, 0, 8) == 0) return 2;
    }
    const char* dot = strrchr(path, '.');
    if (dot && (!strcasecmp(dot, ".jpg") || !strcasecmp(dot, ".jpeg") || !strcasecmp(dot, ".jpe"))) return 1;
    if (dot && !strcasecmp(dot, ".png")) return 2;
    return 0;
}

int pgrt_image_decode(const char* path, int* width, int* height, int* bpp, int* pitch, unsigned char* out,
                      size_t out_size) {
    switch (image_kind(path)) {
        case 1: {
            const int rc = pgrt_jpeg_decode(path, 0, width, height, bpp, pitch, out, out_size);
            if (rc != 0) snprintf(g_err, sizeof g_err, "%s", pgrt_jpeg_error());
            return rc;
        }
        case 2: return pgrt_png_decode(path, width, height, bpp, pitch, out, out_size);
        default: snprintf(g_err, sizeof g_err, "%s: unknown image format (JPEG and PNG are decoded)", path); return -1;
    }
}

const char* pgrt_image_error(void) { return g_err; }
