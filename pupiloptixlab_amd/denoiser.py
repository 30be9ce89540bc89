"""Python mirror of the reference's optix::Denoiser (framework/optix/denoiser.h:7-66)
over the C ABI (pupil_denoiser_*): an edge-avoiding a-trous wavelet filter on
the GPU (csrc/denoise.hip) standing in for the OptiX AI denoiser.

    dn = Denoiser(Denoiser.USE_ALBEDO | Denoiser.USE_NORMAL)
    dn.setup(w, h)
    dn.execute(pt.buffers.get("final result"), out, albedo=pt.buffers.get("albedo"),
               normal=pt.buffers.get("normal"))
"""
from __future__ import annotations

import ctypes as C

from . import abi
from .abi import check, load_library


class Denoiser:
    NONE = 0
    USE_ALBEDO = abi.DENOISE_USE_ALBEDO
    USE_NORMAL = abi.DENOISE_USE_NORMAL
    APPLY_TO_AOV = abi.DENOISE_APPLY_TO_AOV
    USE_TEMPORAL = abi.DENOISE_USE_TEMPORAL
    USE_UPSCALE_2X = abi.DENOISE_USE_UPSCALE_2X
    TILED = abi.DENOISE_TILED

    def __init__(self, mode: int = USE_ALBEDO | USE_NORMAL, device: int = 0):
        self._lib = load_library()
        self._h = C.c_void_p()
        check(self._lib.pupil_denoiser_create(int(device), int(mode), C.byref(self._h)))
        self.mode = int(mode)
        self.sigma_color = 1.0
        self.input_w = self.input_h = 0

    def set_mode(self, mode: int):
        self.mode = int(mode)
        if self.input_w:
            self.setup(self.input_w, self.input_h)

    def setup(self, w: int, h: int, sigma_color: float | None = None):
        if sigma_color is not None:
            self.sigma_color = float(sigma_color)
        check(self._lib.pupil_denoiser_setup(self._h, self.mode, int(w), int(h), self.sigma_color))
        self.input_w, self.input_h = int(w), int(h)

    def execute(self, input, output, albedo=None, normal=None, prev_output=None, stream=None):
        """Tensors on the device: input/output/prev_output (w*h, 4) float32, albedo/normal (w*h, 3)."""
        import torch

        d = abi.DenoiseData()
        d.input = input.data_ptr()
        d.output = output.data_ptr()
        d.prev_output = prev_output.data_ptr() if prev_output is not None else None
        d.albedo = albedo.data_ptr() if albedo is not None else None
        d.normal = normal.data_ptr() if normal is not None else None
        s = stream if stream is not None else torch.cuda.current_stream(input.device)
        check(self._lib.pupil_denoiser_execute(self._h, C.byref(d), C.c_void_p(s.cuda_stream)))

    def close(self):
        if self._h:
            self._lib.pupil_denoiser_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
