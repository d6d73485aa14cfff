/* pgrt_image.h -- texture decode of libpgrt_image.so (pgi_raytracing_amd/csrc/image_jpeg.c).
 *
 * Replaces the FreeImage load in Texture::Texture (APP/texture.cpp:5-54): FreeImage_Load(fif,
 * file, 0) with flags 0 = JPEG_DEFAULT (FreeImage.h:693-695), i.e. IJG libjpeg's fast integer
 * IDCT without fancy upsampling, then FreeImage_ConvertToRawBits(top-down): BGR bytes, rows
 * FreeImage_GetPitch bytes apart -- the layout pgrt_texture (pgrt.h) takes.
 */
#ifndef PGRT_IMAGE_H_
#define PGRT_IMAGE_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dct 0: FreeImage JPEG_DEFAULT (JDCT_IFAST, no fancy upsampling); 1: JPEG_ACCURATE (JDCT_ISLOW,
 * fancy upsampling).  out == NULL: header only (width, height, bpp = 3, pitch).  Returns 0, -1
 * (open / decode error: pgrt_jpeg_error) or -2 (out_size < pitch * height). */
int pgrt_jpeg_decode(const char* path, int dct, int* width, int* height, int* bpp, int* pitch,
                     unsigned char* out, size_t out_size);
const char* pgrt_jpeg_error(void);

/* PNG (lossless: FreeImage's bytes): RGB -> BGR (bpp 3), RGBA -> BGRA (bpp 4), palette / grey
 * expanded to RGB(A), 16-bit samples reduced to 8; FreeImage pitch, top-down.  Same returns. */
int pgrt_png_decode(const char* path, int* width, int* height, int* bpp, int* pitch,
                    unsigned char* out, size_t out_size);
const char* pgrt_png_error(void);

/* Texture::Texture's load (texture.cpp:15-46): the format from the file signature, else the file
 * name (FreeImage_GetFileType / FreeImage_GetFIFFromFilename), then the JPEG_DEFAULT or PNG
 * decode above.  Same returns; pgrt_image_error describes a failure. */
int pgrt_image_decode(const char* path, int* width, int* height, int* bpp, int* pitch,
                      unsigned char* out, size_t out_size);
const char* pgrt_image_error(void);

#ifdef __cplusplus
}
#endif

#endif /* PGRT_IMAGE_H_ */
