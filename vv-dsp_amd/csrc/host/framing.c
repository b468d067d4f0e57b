/* framing.c -- framing helpers on the MI355X backend (C99).
 * The reference's src/core/framing.c:58-146: frame count (host arithmetic),
 * frame fetch and overlap-add (through the shim's kernels), plus batched
 * device-pointer forms of the last two. */
#include "vv_dsp/core/framing.h"
#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp_hip.h"

size_t vv_dsp_get_num_frames(size_t signal_len, size_t frame_len, size_t hop_len, int center) {
    if (hop_len == 0) return 0;
    if (center != 0) return (signal_len + hop_len - 1) / hop_len;
    if (signal_len < frame_len) return 0;
    return 1 + (signal_len - frame_len) / hop_len;
}

vv_dsp_status vv_dsp_fetch_frame(const vv_dsp_real* signal, size_t signal_len, vv_dsp_real* frame_buffer,
                                 size_t frame_len, size_t hop_len, size_t frame_index, int center,
                                 const vv_dsp_real* window) {
    if (!signal || !frame_buffer) return VV_DSP_ERROR_NULL_POINTER;
    if (signal_len == 0 || frame_len == 0 || hop_len == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_fetch_frame_host(signal, signal_len, frame_buffer, frame_len, hop_len, frame_index,
                                                 center, window);
}

vv_dsp_status vv_dsp_overlap_add(const vv_dsp_real* frame, vv_dsp_real* output_signal, size_t output_len,
                                 size_t frame_len, size_t hop_len, size_t frame_index) {
    if (!frame || !output_signal) return VV_DSP_ERROR_NULL_POINTER;
    if (output_len == 0 || frame_len == 0 || hop_len == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_overlap_add_host(frame, output_signal, output_len, frame_len, hop_len, frame_index);
}

vv_dsp_status vv_dsp_fetch_frames_device(const vv_dsp_real* d_signal, size_t signal_len, vv_dsp_real* d_frames,
                                         size_t frame_len, size_t hop_len, size_t frame0, size_t count, int center,
                                         const vv_dsp_real* d_window, void* stream) {
    if (!d_signal || !d_frames) return VV_DSP_ERROR_NULL_POINTER;
    if (signal_len == 0 || frame_len == 0 || hop_len == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_fetch_frames_device(d_signal, signal_len, d_frames, frame_len, hop_len, frame0, count,
                                                    center, d_window, stream);
}

vv_dsp_status vv_dsp_overlap_add_device(const vv_dsp_real* d_frames, size_t count, vv_dsp_real* d_out,
                                        size_t output_len, size_t frame_len, size_t hop_len, size_t frame0,
                                        void* stream) {
    if (!d_frames || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    if (output_len == 0 || frame_len == 0 || hop_len == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_overlap_add_device(d_frames, count, d_out, output_len, frame_len, hop_len, frame0,
                                                   stream);
}
