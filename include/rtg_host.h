/*
 * rtg_host.h — C ABI of the native host side (librtghost.so, raytracer-795_amd/host/):
 * the reference's Parser / Image / renderScene camera loop in C++ above include/rtg.h, so a
 * scene file goes from XML to images without Python (`rtg_cli scene.xml`, the reference's
 * `./raytracer scene.xml`, src/main.cpp:7-14).
 *
 *   rtgh_parse_xml      replaces  new Scene(xml) -> Parser::Parse* (src/Scene.cpp:455-504,
 *                                 src/Parser.h:17-1315) and yields the rtg_scene_desc that
 *                                 rtg_scene_create consumes, plus the cameras
 *   rtgh_save_image     replaces  Image::saveImage (src/Image.cpp:26-107: P3 text when the
 *                                 name contains ".png", else OpenEXR HALF via
 *                                 src/Helper.cpp:361-412)
 *   rtgh_render_scene   replaces  Scene::renderScene (src/Scene.cpp:294-363) end to end
 */
#ifndef RTG_HOST_H_
#define RTG_HOST_H_

#include "rtg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rtgh_scene rtgh_scene;

const char* rtgh_last_error(void);
/* Parse a CENG795 scene file (hw1-hw6 tags plus the hw7 <Renderer>, <RendererParams>,
   <LightSphere>, <LightMesh>).  PLY meshes and image textures are loaded relative to the
   XML's directory.  The descriptor stays valid until rtgh_free. */
int32_t rtgh_parse_xml(const char* xml_path, rtgh_scene** out);
const rtg_scene_desc* rtgh_scene_desc(const rtgh_scene* scene);
int32_t rtgh_num_cameras(const rtgh_scene* scene);
/* Camera i; image_name receives the <ImageName> (truncated to cap-1 bytes). */
int32_t rtgh_camera(const rtgh_scene* scene, int32_t i, rtg_camera_desc* out, char* image_name, int32_t cap);
/* Camera i's hw5 <Tonemap> (Photographic TMO): 1 and *out filled if present, 0 if not. */
int32_t rtgh_camera_tonemap(const rtgh_scene* scene, int32_t i, rtg_tonemap_desc* out);
void rtgh_free(rtgh_scene* scene);

/* Decode an image texture the way the reference's Texture constructor sees it
   (src/Texture.cpp:7-21, 41-74): *rgb = malloc'd ny*nx*3 floats [y][x][c], raw 0..255 for
   PNG/JPEG/PPM, linear floats for OpenEXR (LoadEXR's R,G,B, src/Helper.cpp:346-359).
   Release with rtgh_free_image. */
int32_t rtgh_read_image(const char* path, float** rgb, int32_t* nx, int32_t* ny);
void rtgh_free_image(float* rgb);

/* rgb: ny*nx*3 floats [y][x][c] (Image::_data). */
int32_t rtgh_save_image(const char* name, const float* rgb, int32_t nx, int32_t ny);

/* Parse, build on `device`, render every camera with Philox seed `seed`, save each image
   (under out_dir if not NULL/empty, else at its <ImageName>). */
int32_t rtgh_render_scene(const char* xml_path, int32_t device, uint64_t seed, const char* out_dir);
/* Same, every camera rendered on num_devices GPUs (device, device+1, ...): row-block shards,
   one host thread per GPU, RCCL gather of the rows (rtg_render_opts.num_devices / devices; with
   num_devices = 1 the one GPU is a one-rank RCCL job).  num_devices = 0: rtgh_render_scene. */
int32_t rtgh_render_scene_multi(const char* xml_path, int32_t device, int32_t num_devices, uint64_t seed,
                                const char* out_dir);

#ifdef __cplusplus
}
#endif
#endif /* RTG_HOST_H_ */
