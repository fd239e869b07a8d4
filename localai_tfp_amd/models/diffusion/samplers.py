"""Noise schedules and samplers (the set sd.cpp exposes through the reference's gosd.cpp:27-50:
euler_a, euler, heun, dpm2, dpm++2s_a, dpm++2m, dpm++2mv2, ipndm, ipndm_v, lcm, ddim_trailing, tcd;
schedules default/discrete, karras, exponential, ays, gits).

All samplers are written in the k-diffusion form over a `denoise(x, sigma) -> x0` callable, which
the pipeline builds for either parameterisation:
  * eps models (SD1.x/2.x/SDXL): x_in = x / sqrt(sigma^2 + 1), t = sigma -> discrete timestep,
    x0 = x - sigma * eps
  * rectified-flow models (SD3 / Flux): x_t = (1 - sigma) x0 + sigma * noise, t = 1000 * sigma,
    x0 = x - sigma * v
Ancestral / stochastic steps use the matching noise split for each parameterisation.
"""
from __future__ import annotations

import math

import numpy as np
import torch

SAMPLERS = ("euler_a", "euler", "heun", "dpm2", "dpm++2s_a", "dpm++2m", "dpm++2mv2", "ipndm", "ipndm_v", "lcm",
            "ddim_trailing", "tcd")
SCHEDULES = ("default", "discrete", "karras", "exponential", "ays", "gits")


# ------------------------------------------------------------------------------------------------
# schedules

def sd_alphas_cumprod(n: int = 1000, beta_start: float = 0.00085, beta_end: float = 0.012) -> np.ndarray:
    betas = np.linspace(beta_start ** 0.5, beta_end ** 0.5, n, dtype=np.float64) ** 2
    return np.cumprod(1.0 - betas)


class EpsSchedule:
    """Discrete DDPM schedule of the SD UNets (scaled-linear betas)."""

    def __init__(self):
        ac = sd_alphas_cumprod()
        self.sigmas = np.sqrt((1 - ac) / ac)
        self.log_sigmas = np.log(self.sigmas)

    @property
    def sigma_min(self):
        return float(self.sigmas[0])

    @property
    def sigma_max(self):
        return float(self.sigmas[-1])

    def t_of(self, sigma: float) -> float:
        ls = math.log(max(sigma, 1e-10))
        return float(np.interp(ls, self.log_sigmas, np.arange(len(self.sigmas))))

    def sigma_of(self, t: float) -> float:
        return float(np.exp(np.interp(t, np.arange(len(self.sigmas)), self.log_sigmas)))


class FlowSchedule:
    """Rectified-flow schedule (SD3: shift 3.0) with sigma in (0, 1]."""

    def __init__(self, shift: float = 3.0):
        self.shift = shift

    sigma_min = 0.0
    sigma_max = 1.0

    def sigma_of(self, t: float) -> float:  # t in [0, 1000]
        s = t / 1000.0
        return self.shift * s / (1 + (self.shift - 1) * s)

    def t_of(self, sigma: float) -> float:
        return sigma * 1000.0


def get_sigmas(sched, steps: int, kind: str = "default") -> list[float]:
    """Descending sigmas of length steps + 1, ending in 0."""
    kind = kind or "default"
    flow = isinstance(sched, FlowSchedule)
    if kind in ("default", "discrete", "ays", "gits") or flow and kind != "karras":
        if flow:
            ts = np.linspace(1000.0, 1000.0 / steps, steps) if steps > 0 else np.array([])
            sig = [sched.sigma_of(t) for t in ts]
        else:
            ts = np.linspace(999.0, 0.0, steps)
            sig = [sched.sigma_of(t) for t in ts]
        return sig + [0.0]
    lo = max(sched.sigma_min, 1e-3) if flow else sched.sigma_min
    hi = sched.sigma_max
    if kind == "karras":
        rho = 7.0
        r = np.linspace(0, 1, steps)
        sig = (hi ** (1 / rho) + r * (lo ** (1 / rho) - hi ** (1 / rho))) ** rho
    elif kind == "exponential":
        sig = np.exp(np.linspace(math.log(hi), math.log(lo), steps))
    else:
        raise ValueError(f"unknown schedule {kind!r}")
    return [float(s) for s in sig] + [0.0]


# ------------------------------------------------------------------------------------------------
# samplers

def _noise_like(x, gen):
    return torch.randn(x.shape, generator=gen, device=x.device, dtype=torch.float32)


def _ancestral(sigma, sigma_next, flow: bool, eta: float = 1.0):
    """-> (sigma_down, sigma_up, alpha_scale) for one ancestral step."""
    if sigma_next == 0:
        return 0.0, 0.0, 1.0
    if not flow:
        up = min(sigma_next, eta * math.sqrt(max(0.0, sigma_next ** 2 * (sigma ** 2 - sigma_next ** 2) / sigma ** 2)))
        return math.sqrt(max(0.0, sigma_next ** 2 - up ** 2)), up, 1.0
    # rectified flow: x = (1-s) x0 + s n; renoise with the right mixture
    down = sigma_next * (1 + (sigma_next / sigma - 1) * eta)
    alpha_ip1, alpha_down = 1 - sigma_next, 1 - down
    up = math.sqrt(max(0.0, sigma_next ** 2 - down ** 2 * alpha_ip1 ** 2 / alpha_down ** 2))
    return down, up, alpha_ip1 / alpha_down


def sample(denoise, x: torch.Tensor, sigmas: list[float], sampler: str = "euler", flow: bool = False,
           generator=None, callback=None) -> torch.Tensor:
    sampler = (sampler or "euler").lower()
    n = len(sigmas) - 1
    old_d = None
    old_x0 = None
    ds_hist: list[torch.Tensor] = []
    for i in range(n):
        s, sn = sigmas[i], sigmas[i + 1]
        x0 = denoise(x, s)
        d = (x - x0) / s
        if sampler == "euler" or (sampler in ("heun", "dpm2") and sn == 0):
            x = x + d * (sn - s)
        elif sampler == "heun":
            x2 = x + d * (sn - s)
            d2 = (x2 - denoise(x2, sn)) / sn
            x = x + (d + d2) / 2 * (sn - s)
        elif sampler == "dpm2":
            sm = math.exp((math.log(s) + math.log(sn)) / 2)
            x2 = x + d * (sm - s)
            d2 = (x2 - denoise(x2, sm)) / sm
            x = x + d2 * (sn - s)
        elif sampler in ("euler_a", "dpm++2s_a"):
            down, up, a = _ancestral(s, sn, flow)
            if sampler == "euler_a" or down == 0:
                x = x + d * (down - s)
            else:  # DPM-Solver++(2S) ancestral
                t, tn = -math.log(s), -math.log(down)
                h = tn - t
                sm = math.exp(-(t + 0.5 * h))
                x2 = (sm / s) * x - math.expm1(-0.5 * h) * x0
                x0b = denoise(x2, sm)
                x = (down / s) * x - math.expm1(-h) * x0b
            if sn > 0:
                x = a * x + _noise_like(x, generator) * up
        elif sampler in ("dpm++2m", "dpm++2mv2"):
            t, tn = -math.log(s), -math.log(sn) if sn > 0 else float("inf")
            h = tn - t
            if old_x0 is None or sn == 0:
                x = (sn / s) * x - math.expm1(-h) * x0 if sn > 0 else x0
            else:
                h_last = t - (-math.log(sigmas[i - 1]))
                r = h_last / h
                if sampler == "dpm++2mv2":
                    r = max(r, 1e-3)
                xd = (1 + 1 / (2 * r)) * x0 - (1 / (2 * r)) * old_x0
                x = (sn / s) * x - math.expm1(-h) * xd
            old_x0 = x0
        elif sampler in ("ipndm", "ipndm_v"):
            ds_hist.append(d)
            k = len(ds_hist)
            if k == 1:
                dd = d
            elif k == 2:
                dd = (3 * ds_hist[-1] - ds_hist[-2]) / 2
            elif k == 3:
                dd = (23 * ds_hist[-1] - 16 * ds_hist[-2] + 5 * ds_hist[-3]) / 12
            else:
                dd = (55 * ds_hist[-1] - 59 * ds_hist[-2] + 37 * ds_hist[-3] - 9 * ds_hist[-4]) / 24
            ds_hist = ds_hist[-3:]
            x = x + dd * (sn - s)
        elif sampler in ("lcm", "tcd"):
            x = x0
            if sn > 0:
                n_ = _noise_like(x, generator)
                x = (1 - sn) * x0 + sn * n_ if flow else x0 + sn * n_
        elif sampler == "ddim_trailing":
            if sn == 0:
                x = x0
            else:
                eps = d  # (x - x0) / sigma
                x = (1 - sn) * x0 + sn * (x - (1 - s) * x0) / s if flow else x0 + sn * eps
        else:
            raise ValueError(f"unknown sampler {sampler!r} (supported: {', '.join(SAMPLERS)})")
        old_d = d
        if callback is not None:
            callback(i, x)
    del old_d
    return x
