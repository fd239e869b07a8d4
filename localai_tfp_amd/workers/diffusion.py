"""Image generation worker: the reference's `stablediffusion-ggml` (sd.cpp, gosd.cpp/gosd.go) and
`diffusers` backends behind one GenerateImage RPC.

LoadModel: a diffusers-layout SD3 directory (MMDiT), Flux.1 directory (FluxTransformer2DModel) or
SD1.x / SD2.x / SDXL directory (UNet; a StableDiffusionDepth2ImgPipeline directory — 5-channel UNet plus
depth_estimator/ — runs depth-to-image with `src` as the source image, synthetic: `sd2-depth-test`); a stable-diffusion.cpp-style single file (.safetensors / .ckpt /
GGUF: Flux.1 in BFL names, SD1.x / SD2.x / SDXL in LDM/SGM names) with the component options
clip_l_path / clip_g_path / t5xxl_path / vae_path (models/diffusion/single_file.py); or `synthetic:sd3-medium | sd3-medium-no-t5 | sd3-test | sd15 |
sdxl | sd15-test | sdxl-test | flux-dev | flux-schnell | flux-test` (random-init weights). For Flux,
cfg_scale is the distilled guidance (default 3.5). ModelOptions.Options ("key:value", as gosd.cpp:56-162 parses them):
  sampler:<euler|euler_a|heun|dpm2|dpm++2s_a|dpm++2m|dpm++2mv2|ipndm|ipndm_v|lcm|ddim_trailing|tcd>
  scheduler:<default|discrete|karras|exponential|ays|gits>
  cfg_scale:<float>   (ModelOptions.CFGScale also honoured)
  t5:<true|false>     (drop the T5-XXL encoder; SD3 runs with zero T5 features)
  strength:<float>    (img2img denoise strength)
LoRA: LoraAdapter (+LoraScale) and LoraAdapters (+LoraScales) — kohya or diffusers/PEFT safetensors —
are merged into the weights at load (models/diffusion/lora.py). ControlNet (UNet pipelines): a diffusers
ControlNetModel directory or `synthetic`; with it set, `src` is the control image (option control_scale).
GenerateImage: positive / negative prompt, width, height, step, seed, dst (PNG), src (img2img).
Video (models/diffusion/svd.py): PipelineType StableVideoDiffusionPipeline (or `synthetic:svd | svd-xt |
svd-test`, or a directory whose model_index.json names that pipeline) loads Stable Video Diffusion;
GenerateImage with src = start image, or GenerateVideo (start_image, width, height, num_frames, fps, seed,
cfg_scale = max guidance), writes the clip to dst (MP4 Motion-JPEG, or .gif / .webp). Options: steps, fps,
motion_bucket_id, noise_aug_strength, min_guidance_scale, max_guidance_scale, decode_chunk_size.
One image per call; data parallelism = one worker replica per GPU (model config `data_parallel`),
with the gateway spreading concurrent requests across replicas.
"""
from __future__ import annotations

import logging
import os

from ..grpc import pb
from ..grpc.server import BackendServicer, worker_main

log = logging.getLogger("localai_tfp_amd.workers.diffusion")


class DiffusionServicer(BackendServicer):
    locking = True  # one generation at a time per GPU (gosd.go SingleThread)

    def __init__(self, device: str | None = None):
        super().__init__()
        self.device = device
        self.pipe = None
        self.defaults = {}

    def LoadModel(self, request, context):
        import torch
        from ..models.diffusion.pipeline import SD3Pipeline
        try:
            if self.device is None:
                self.device = "cuda:0" if torch.cuda.is_available() else "cpu"
            opts = {}
            for kv in request.Options:
                k, _, v = kv.partition(":")
                opts[k.strip()] = v.strip()
            use_t5 = opts.get("t5", "true").lower() not in ("0", "false", "no")
            from ..models.diffusion import flux as FX
            from ..models.diffusion import sd_pipeline as U
            path = request.ModelFile or request.Model
            from ..models.diffusion import svd as SV
            if _is_svd(request, path):
                if path.startswith("synthetic:"):
                    self.pipe = SV.SVDPipeline.synthetic(path.split(":", 1)[1] or "svd-xt", self.device)
                else:
                    if not os.path.isabs(path) and request.ModelPath:
                        path = os.path.join(request.ModelPath, path)
                    self.pipe = SV.SVDPipeline.from_diffusers(path, self.device)
                self.defaults = dict(steps=int(opts.get("steps", 25)), fps=int(opts.get("fps", 7)),
                                     motion_bucket_id=int(opts.get("motion_bucket_id", 127)),
                                     noise_aug_strength=float(opts.get("noise_aug_strength", 0.02)),
                                     min_guidance=float(opts.get("min_guidance_scale", 1.0)),
                                     max_guidance=float(opts.get("max_guidance_scale", request.CFGScale or 3.0)),
                                     decode_chunk=int(opts.get("decode_chunk_size", 8)))
                return pb.Result(message="loaded", success=True)
            from ..models.diffusion import lumina2 as LU
            pcls = _pipeline_class(request, path)
            if path.startswith("synthetic:"):
                name = path.split(":", 1)[1]
                if not use_t5 and name == "sd3-medium":
                    name = "sd3-medium-no-t5"
                if name.startswith("lumina2"):
                    self.pipe = LU.Lumina2Pipeline.synthetic(name, self.device)
                elif name.startswith("sana"):
                    from ..models.diffusion.sana import SanaPipeline
                    self.pipe = SanaPipeline.synthetic(name, self.device)
                elif name in U.PRESETS:  # SD1.x / SDXL UNet models
                    self.pipe = U.UNetPipeline.synthetic(name, self.device)
                elif name.startswith("flux"):
                    self.pipe = FX.FluxPipeline.synthetic(name, self.device)
                else:
                    self.pipe = SD3Pipeline.synthetic(name, self.device)
            else:
                if not os.path.isabs(path) and request.ModelPath:
                    path = os.path.join(request.ModelPath, path)
                if os.path.isfile(path):
                    # stable-diffusion.cpp-style single file / GGUF + component files (gosd.cpp:56-162)
                    from ..models.diffusion.single_file import from_single_file

                    def comp(k):
                        v = opts.get(k, "")
                        return os.path.join(request.ModelPath, v) if v and not os.path.isabs(v) and request.ModelPath else v
                    self.pipe = from_single_file(path, self.device, {k: comp(k) for k in (
                        "clip_l_path", "clip_g_path", "t5xxl_path", "vae_path")})
                elif not os.path.isdir(path):
                    raise ValueError(f"{path}: expected a model file or a diffusers-layout model directory")
                elif pcls.startswith("Lumina2"):  # Lumina2Text2ImgPipeline / Lumina2Pipeline (backend.py:213-216)
                    self.pipe = LU.Lumina2Pipeline.from_diffusers(path, self.device)
                elif pcls.startswith("Sana"):  # SanaPipeline (backend.py:218-221)
                    from ..models.diffusion.sana import SanaPipeline
                    self.pipe = SanaPipeline.from_diffusers(path, self.device)
                elif os.path.isdir(os.path.join(path, "unet")):
                    self.pipe = U.UNetPipeline.from_diffusers(path, self.device)
                elif _is_flux(path):
                    self.pipe = FX.FluxPipeline.from_diffusers(path, self.device)
                else:
                    self.pipe = SD3Pipeline.from_diffusers(path, self.device, use_t5=use_t5)
            if request.ControlNet:
                if not isinstance(self.pipe, U.UNetPipeline):
                    raise ValueError("ControlNet is supported with SD1.x / SD2.x / SDXL UNet pipelines")
                cpath = request.ControlNet
                if not cpath.startswith("synthetic") and not os.path.isabs(cpath) and request.ModelPath:
                    cpath = os.path.join(request.ModelPath, cpath)
                self.pipe.set_controlnet(cpath)
            adapters = _lora_list(request)
            if adapters:
                from ..models.diffusion.lora import apply_adapters
                apply_adapters(self.pipe, adapters)
            sampler, schedule = opts.get("sampler", "euler"), opts.get("scheduler", "default")
            if request.SchedulerType:
                sampler, schedule = diffusers_scheduler(request.SchedulerType)
            self.defaults = dict(sampler=sampler, schedule=schedule,
                                 cfg_scale=float(opts.get("cfg_scale", request.CFGScale or
                                                          (3.5 if isinstance(self.pipe, FX.FluxPipeline) else
                                                           4.0 if isinstance(self.pipe, LU.Lumina2Pipeline) else
                                                           4.5 if type(self.pipe).__name__ == "SanaPipeline" else 7.0))),
                                 strength=float(opts.get("strength", 0.75)),
                                 control_scale=float(opts.get("control_scale", 1.0)))
            return pb.Result(message="loaded", success=True)
        except Exception as ex:
            log.exception("LoadModel failed")
            return pb.Result(message=f"failed to load model: {ex}", success=False)

    def _video(self, src: str, dst: str, width: int, height: int, frames: int, fps: int, seed: int,
               cfg_scale: float):
        from PIL import Image

        from ..models.diffusion.svd import VideoParams
        from ..utils.video import write_video
        if not src:
            raise ValueError("image-to-video needs a start image (src / start_image)")
        d = self.defaults
        vp = VideoParams(width=width or 1024, height=height or 576, num_frames=frames, steps=d["steps"],
                         fps=fps or d["fps"], motion_bucket_id=d["motion_bucket_id"],
                         noise_aug_strength=d["noise_aug_strength"], min_guidance=d["min_guidance"],
                         max_guidance=cfg_scale or d["max_guidance"], seed=seed, decode_chunk=d["decode_chunk"])
        with Image.open(src) as im:
            out = self.pipe.generate(im.convert("RGB"), vp)
        write_video(out, dst, fps=vp.fps)

    def GenerateVideo(self, request, context):
        """backend.proto GenerateVideoRequest (core/backend/video.go:22): start_image -> video at dst."""
        from ..models.diffusion.svd import SVDPipeline
        if not isinstance(self.pipe, SVDPipeline):
            return pb.Result(message="this model does not generate video (load a StableVideoDiffusionPipeline)",
                             success=False)
        try:
            self._video(request.start_image, request.dst, request.width, request.height, request.num_frames,
                        request.fps, request.seed, request.cfg_scale)
            return pb.Result(message="Media generated successfully", success=True)
        except Exception as ex:
            log.exception("GenerateVideo failed")
            return pb.Result(message=f"generation failed: {ex}", success=False)

    def GenerateImage(self, request, context):
        from ..models.diffusion.pipeline import GenParams, load_image, save_png
        from ..models.diffusion.svd import SVDPipeline
        if self.pipe is None:
            return pb.Result(message="model not loaded", success=False)
        if isinstance(self.pipe, SVDPipeline):  # img2vid through GenerateImage (backend.py:338-341)
            try:
                self._video(request.src, request.dst, request.width, request.height, 0, 0, request.seed, 0.0)
                return pb.Result(message="Media generated successfully", success=True)
            except Exception as ex:
                log.exception("img2vid failed")
                return pb.Result(message=f"generation failed: {ex}", success=False)
        try:
            w = request.width or 512
            h = request.height or 512
            gp = GenParams(width=w, height=h, steps=request.step or 20, seed=request.seed,
                           negative=request.negative_prompt,
                           **{k: v for k, v in self.defaults.items() if k != "control_scale"})
            gp.extra["clip_skip"] = request.CLIPSkip
            init = load_image(request.src, w, h) if request.src else None
            if init is not None and getattr(self.pipe, "controlnet", None) is not None:
                gp.extra["control_image"], init = init, None  # src is the control image (backend.py:309-312)
                gp.extra["control_scale"] = self.defaults.get("control_scale", 1.0)
            img = self.pipe.generate(request.positive_prompt, gp, init)
            save_png(img, request.dst)
            return pb.Result(message="ok", success=True)
        except Exception as ex:
            log.exception("GenerateImage failed")
            return pb.Result(message=f"generation failed: {ex}", success=False)


def _lora_list(request) -> list[tuple[str, float]]:
    """LoraAdapter (+LoraScale, default 1) and LoraAdapters (+LoraScales), relative to ModelPath."""
    def full(p):
        return p if os.path.isabs(p) or not request.ModelPath else os.path.join(request.ModelPath, p)
    out = []
    if request.LoraAdapter:
        out.append((full(request.LoraAdapter), request.LoraScale or 1.0))
    scales = list(request.LoraScales)
    for i, p in enumerate(request.LoraAdapters):
        out.append((full(p), scales[i] if i < len(scales) else 1.0))
    return out


def _is_svd(request, path: str) -> bool:
    """StableVideoDiffusionPipeline by pipeline type, synthetic preset name or model_index.json."""
    import json
    if request.PipelineType == "StableVideoDiffusionPipeline":
        return True
    if path.startswith("synthetic:"):
        return path.split(":", 1)[1].startswith("svd")
    try:
        with open(os.path.join(path if os.path.isabs(path) else os.path.join(request.ModelPath or "", path),
                               "model_index.json")) as f:
            return json.load(f).get("_class_name") == "StableVideoDiffusionPipeline"
    except (OSError, ValueError):
        return False


def _pipeline_class(request, path: str) -> str:
    """The request's PipelineType, else model_index.json's _class_name of a diffusers directory ("" if none)."""
    import json
    if request.PipelineType:
        return request.PipelineType
    if path.startswith("synthetic:"):
        return ""
    try:
        with open(os.path.join(path if os.path.isabs(path) else os.path.join(request.ModelPath or "", path),
                               "model_index.json")) as f:
            return str(json.load(f).get("_class_name") or "")
    except (OSError, ValueError):
        return ""


def _is_flux(path: str) -> bool:
    import json
    try:
        with open(os.path.join(path, "transformer", "config.json")) as f:
            return "num_single_layers" in json.load(f)
    except OSError:
        return False


def main(argv=None):
    worker_main(DiffusionServicer, argv)


if __name__ == "__main__":
    main()


# diffusers SchedulerType names of the reference (backend/python/diffusers/backend.py:81-133) -> this
# framework's k-diffusion-style samplers (models/diffusion/samplers.py); a "k_" prefix selects Karras sigmas
# like use_karras_sigmas. Exact for euler / euler_a / heun / dpm_2 / dpmpp_2m; the rest map to the
# same-order sampler of the family (parity with diffusers' implementations unpinned: not importable here).
DIFFUSERS_SCHEDULERS = {
    "euler": "euler", "euler_a": "euler_a", "heun": "heun", "dpm_2": "dpm2", "dpmpp_2m": "dpm++2m",
    "ddim": "ddim_trailing", "pndm": "ipndm", "lms": "ipndm", "unipc": "dpm++2m", "dpm_2_a": "dpm++2s_a",
    "dpmpp_sde": "dpm++2s_a", "dpmpp_2m_sde": "dpm++2m",
}


def diffusers_scheduler(name: str) -> tuple[str, str]:
    n = (name or "").strip().lower()
    karras = n.startswith("k_")
    if karras:
        n = n[2:]
    if n not in DIFFUSERS_SCHEDULERS:
        raise ValueError(f"Invalid scheduler {name!r} (have {sorted(DIFFUSERS_SCHEDULERS)} and k_ variants)")
    return DIFFUSERS_SCHEDULERS[n], ("karras" if karras else "default")
