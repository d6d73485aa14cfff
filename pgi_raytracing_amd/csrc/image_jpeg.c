/* image_jpeg.c -- JPEG texture decode as the reference's FreeImage gets it (libpgrt_image.so).
 *
 * Texture::Texture (APP/texture.cpp:5-54) calls FreeImage_Load(fif, file, 0): flags 0 is
 * JPEG_DEFAULT, "loading (see JPEG_FAST)" (FreeImage.h:693-695).  FreeImage 3.18's JPEG plugin
 * (PluginJPEG.cpp, not vendored in the reference) decodes with its bundled IJG libjpeg 9c and,
 * unless JPEG_ACCURATE is set, selects the fast integer IDCT (dct_method = JDCT_IFAST) and turns
 * fancy (smoothed) chroma upsampling off.  FreeImage_ConvertToRawBits(..., topdown = TRUE)
 * then hands the texture its pixels as BGR bytes, top row first, rows FreeImage_GetPitch bytes
 * apart (width * 3 rounded up to 4).
 *
 * Here: the same IJG decoder with the same two settings (libjpeg 9, /opt/conda/lib/libjpeg.so.9
 * in this image), written in exactly that layout.  Greyscale JPEGs are expanded to BGR
 * (FreeImage would keep 8 bpp; no reference asset is greyscale).  Plain C ABI, used by the
 * Python scene loader (pgi_raytracing_amd/scene.py) and the texture sidecar tool.
 */
#include <setjmp.h>
#include <stdio.h>
#include <string.h>

#include <jpeglib.h>

#include "pgrt_image.h"

struct err_mgr {
    struct jpeg_error_mgr pub;
    jmp_buf jb;
    char msg[JMSG_LENGTH_MAX];
};

static void on_error(j_common_ptr c) {
    struct err_mgr* e = (struct err_mgr*)c->err;
    (*c->err->format_message)(c, e->msg);
    longjmp(e->jb, 1);
}

static char g_err[JMSG_LENGTH_MAX + 64];

const char* pgrt_jpeg_error(void) { return g_err; }

/* dct: 0 = FreeImage JPEG_DEFAULT (JDCT_IFAST, no fancy upsampling); 1 = JDCT_ISLOW with fancy
 * upsampling (JPEG_ACCURATE; for cross-checks only).  out == NULL: header only.  Returns 0, or
 * -1 (open / decode error, pgrt_jpeg_error) / -2 (out_size too small). */
int pgrt_jpeg_decode(const char* path, int dct, int* width, int* height, int* bpp, int* pitch, unsigned char* out,
                     size_t out_size) {
    struct jpeg_decompress_struct ci;
    struct err_mgr em;
    FILE* f = fopen(path, "rb");
    g_err[0] = 0;
    if (!f) {
        snprintf(g_err, sizeof g_err, "cannot open %s", path);
        return -1;
    }
    ci.err = jpeg_std_error(&em.pub);
    em.pub.error_exit = on_error;
    if (setjmp(em.jb)) {
        snprintf(g_err, sizeof g_err, "%s: %s", path, em.msg);
        jpeg_destroy_decompress(&ci);
        fclose(f);
        return -1;
    }
    jpeg_create_decompress(&ci);
    jpeg_stdio_src(&ci, f);
    jpeg_read_header(&ci, TRUE);
    ci.out_color_space = JCS_RGB;
    if (dct == 0) {
        ci.dct_method = JDCT_IFAST;
        ci.do_fancy_upsampling = FALSE;
    } else {
        ci.dct_method = JDCT_ISLOW;
        ci.do_fancy_upsampling = TRUE;
    }
    jpeg_calc_output_dimensions(&ci);
    const int w = (int)ci.output_width, h = (int)ci.output_height;
    const int p = ((w * 24 + 31) / 32) * 4; /* FreeImage_GetPitch */
    *width = w;
    *height = h;
    *bpp = 3;
    *pitch = p;
    if (!out) {
        jpeg_destroy_decompress(&ci);
        fclose(f);
        return 0;
    }
    if (out_size < (size_t)p * (size_t)h) {
        jpeg_destroy_decompress(&ci);
        fclose(f);
        snprintf(g_err, sizeof g_err, "%s: output buffer too small", path);
        return -2;
    }
    memset(out, 0, (size_t)p * (size_t)h);
    jpeg_start_decompress(&ci);
    while (ci.output_scanline < ci.output_height) {
        unsigned char* row = out + (size_t)ci.output_scanline * (size_t)p;
        JSAMPROW rp = row;
        jpeg_read_scanlines(&ci, &rp, 1);
        for (int x = 0; x < w; ++x) { /* RGB -> BGR in place */
            unsigned char t = row[3 * x];
            row[3 * x] = row[3 * x + 2];
            row[3 * x + 2] = t;
        }
    }
    jpeg_finish_decompress(&ci);
    jpeg_destroy_decompress(&ci);
    fclose(f);
    return 0;
}
