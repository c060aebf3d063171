/* vge_ingest.h -- on-disk feature ingest for the AC/TC scoring path.
 *
 * Host-only C ABI (no HIP types), exported by libvge.so.  Replaces the reference's per-video readers:
 *   np.load(<video>.npz) -> pose [T,23,3,3], global_orient [T,1,3,3], betas [T,10], vit [T,Dv]
 *                                               (utils.py:383-409 WindowDataset._try_one; the npz is
 *                                                extract_mesh.py:35-43's np.savez_compressed output)
 *   np.load(<kp_dir>/.../keypoints.npy) -> [T',120]        (utils.py:410-424)
 * as a multithreaded native decoder: the zip central directory is parsed (zip64 included), each member
 * is raw-deflate inflated (zlib) straight into caller-provided -- typically pinned -- host buffers at
 * the frame-store offsets the GPU path uses (vge.data.FrameStore / vge_frame_store), with no Python
 * objects or intermediate copies per array.  float64 members are converted to float32 (the reference
 * feeds float32 tensors to the model).
 *
 * Two calls per set of videos:
 *   vge_ingest_probe  -- shapes from the npy headers only (inflates the first few hundred bytes of
 *                        two members per file); the caller lays out the frame store from them
 *   vge_ingest_decode -- full decode into the laid-out buffers
 * Per-video failures are reported per video (status[i]), so the Python driver can mirror the
 * reference's error behaviour: an unreadable npz is skipped with a message (eval.py:93-95), a missing
 * keypoint file raises in the scoring path (utils.py:416-417) and is tolerated for the stats
 * (utils.py:669-678).
 */
#ifndef VGE_INGEST_H
#define VGE_INGEST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-video status codes (also the return value of the calls: VGE_OK or the first failure) */
enum {
  VGE_INGEST_OK = 0,
  VGE_INGEST_ERR_ARG = 1,         /* bad argument */
  VGE_INGEST_ERR_IO = 7,          /* npz unreadable / malformed (not a zip, missing member, bad npy) */
  VGE_INGEST_ERR_SHAPE = 8,       /* a member's shape disagrees with the layout (pose/gori/betas/vit T, dims) */
  VGE_INGEST_ERR_KP = 9           /* keypoints.npy present but unreadable / not [T',120] */
};

typedef struct {
  int32_t n_frames;  /* pose.shape[0] */
  int32_t vit_dim;   /* vit.shape[1] */
  int32_t kp_frames; /* keypoints.npy rows; -1 when kp_paths[i] is NULL or the file does not exist */
  int32_t status;    /* VGE_INGEST_OK or an error code above */
} vge_clip_info;

/* npz_paths[n]; kp_paths[n] (entries may be NULL; kp_paths itself may be NULL).  n_threads <= 0:
 * vge_ingest_default_threads().  Fills info[n]; returns VGE_INGEST_OK if every video probed cleanly, else the
 * first failing video's code (the others are still probed). */
/* Thread count the calls use when n_threads <= 0: VGE_INGEST_THREADS, else OMP_NUM_THREADS if > 1, else
 * the process's CPU share (cgroup quota / affinity mask) divided by LOCAL_WORLD_SIZE; at most 64. */
int vge_ingest_default_threads(void);

int vge_ingest_probe(const char* const* npz_paths, const char* const* kp_paths, int n, int n_threads,
                     vge_clip_info* info);

/* Decode video i into rows [videos[4i], videos[4i] + videos[4i+1]) of pose [*,207], gori [*,9],
 * betas [*,10], vit [*,vit_dim] and, when videos[4i+3] > 0, rows [videos[4i+2], +videos[4i+3]) of
 * kp [*,120].  videos[4i+1] must equal the file's T (and videos[4i+3] its T').  status[n] (may be NULL)
 * receives the per-video codes. */
int vge_ingest_decode(const char* const* npz_paths, const char* const* kp_paths, int n, int n_threads,
                      const int32_t* videos, int vit_dim, float* pose, float* gori, float* betas, float* vit,
                      float* kp, int32_t* status);

#ifdef __cplusplus
}
#endif
#endif /* VGE_INGEST_H */
