/* framing.h -- signal framing and overlap-add (reference include/vv_dsp/core.h:
 * 460-530, implemented in src/core/framing.c:58-146).  Same signatures and
 * semantics; the MI355X library runs the frame copy and the accumulation on
 * the GPU (batched forms in vv_dsp/vv_dsp_amd.h). */
#ifndef VV_DSP_CORE_FRAMING_H
#define VV_DSP_CORE_FRAMING_H
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif
/* center == 0: 1 + (signal_len - frame_len) / hop_len (0 if signal_len < frame_len);
 * center != 0: ceil(signal_len / hop_len).  0 when hop_len == 0. */
size_t vv_dsp_get_num_frames(size_t signal_len, size_t frame_len, size_t hop_len, int center);
/* frame_index's frame: starts at frame_index*hop_len (center: minus frame_len/2);
 * zero padding outside the signal, or reflection about its ends when center;
 * times window[i] when window != NULL */
vv_dsp_status vv_dsp_fetch_frame(const vv_dsp_real* signal, size_t signal_len, vv_dsp_real* frame_buffer,
                                 size_t frame_len, size_t hop_len, size_t frame_index, int center,
                                 const vv_dsp_real* window);
/* output_signal[frame_index*hop_len + i] += frame[i] for indices below output_len */
vv_dsp_status vv_dsp_overlap_add(const vv_dsp_real* frame, vv_dsp_real* output_signal, size_t output_len,
                                 size_t frame_len, size_t hop_len, size_t frame_index);
#ifdef __cplusplus
}
#endif
#endif
