"""Textbook step-by-step samplers (the round-1 implementation, one torch op at a time): the
oracle that the generic fused-sampler coefficients (arbius_amd/models/schedulers.py StepPlan,
ops/csrc/sampler.hip) are checked against in tests/test_samplers.py."""

from __future__ import annotations

import math
from typing import List, Optional

import numpy as np
import torch


def sd_alphas_cumprod(n_train=1000, beta_start=0.00085, beta_end=0.012, schedule="scaled_linear"):
    if schedule == "scaled_linear":
        betas = np.linspace(beta_start ** 0.5, beta_end ** 0.5, n_train, dtype=np.float64) ** 2
    elif schedule == "linear":
        betas = np.linspace(beta_start, beta_end, n_train, dtype=np.float64)
    elif schedule == "cosine":
        s = 0.008
        steps = np.arange(n_train + 1, dtype=np.float64) / n_train
        f = np.cos((steps + s) / (1 + s) * math.pi / 2) ** 2
        betas = np.clip(1 - f[1:] / f[:-1], 0, 0.999)
    else:
        raise ValueError(schedule)
    return np.cumprod(1.0 - betas)


class Scheduler:
    name = "base"
    init_noise_sigma = 1.0
    needs_noise = False

    def __init__(self, steps: int, n_train: int = 1000, alphas_cumprod=None):
        self.steps = steps
        self.n_train = n_train
        self.ac = sd_alphas_cumprod(n_train) if alphas_cumprod is None else np.asarray(alphas_cumprod)
        self.timesteps: List[float] = []

    def scale_model_input(self, x, i):
        return x

    def step(self, eps, i, x, generator: Optional[torch.Generator] = None):
        raise NotImplementedError

    def _leading(self, offset=1):
        ratio = self.n_train // self.steps
        return [int(v) for v in (np.arange(0, self.steps) * ratio).round()[::-1] + offset]


class DDIM(Scheduler):
    name = "DDIM"

    def __init__(self, steps, eta=0.0, **kw):
        super().__init__(steps, **kw)
        self.eta = eta
        self.timesteps = self._leading(1)
        self.ratio = self.n_train // steps
        self.needs_noise = eta > 0

    def step(self, eps, i, x, generator=None):
        t = self.timesteps[i]
        tp = t - self.ratio
        a_t = float(self.ac[t])
        a_p = float(self.ac[tp]) if tp >= 0 else float(self.ac[0])
        x0 = (x - math.sqrt(1 - a_t) * eps) / math.sqrt(a_t)
        var = (1 - a_p) / (1 - a_t) * (1 - a_t / a_p)
        std = self.eta * math.sqrt(max(var, 0.0))
        out = math.sqrt(a_p) * x0 + math.sqrt(max(1 - a_p - std * std, 0.0)) * eps
        if std > 0:
            out = out + std * _randn_like(x, generator)
        return out


def _randn_like(x, generator):
    n = torch.randn(x.shape, generator=generator, dtype=torch.float32, device="cpu")
    return n.to(x.device)


class _Sigma(Scheduler):
    """Karras-style samplers in sigma space (K_EULER, K_EULER_ANCESTRAL, KLMS)."""

    def __init__(self, steps, **kw):
        super().__init__(steps, **kw)
        ts = np.linspace(0, self.n_train - 1, steps, dtype=np.float64)[::-1].copy()
        all_s = np.sqrt((1 - self.ac) / self.ac)
        sig = np.interp(ts, np.arange(len(all_s)), all_s)
        self.sigmas = np.concatenate([sig, [0.0]])
        self.timesteps = [float(v) for v in ts]
        self.init_noise_sigma = float(math.sqrt(self.sigmas.max() ** 2 + 1))

    def scale_model_input(self, x, i):
        return x / math.sqrt(self.sigmas[i] ** 2 + 1)


class EulerDiscrete(_Sigma):
    name = "K_EULER"

    def step(self, eps, i, x, generator=None):
        s, sn = self.sigmas[i], self.sigmas[i + 1]
        return x + eps * (sn - s)


class EulerAncestral(_Sigma):
    name = "K_EULER_ANCESTRAL"
    needs_noise = True

    def step(self, eps, i, x, generator=None):
        s, sn = self.sigmas[i], self.sigmas[i + 1]
        up = math.sqrt(max(sn ** 2 * (s ** 2 - sn ** 2) / s ** 2, 0.0))
        down = math.sqrt(max(sn ** 2 - up ** 2, 0.0))
        x = x + eps * (down - s)
        if up > 0:
            x = x + _randn_like(x, generator) * up
        return x


class LMSDiscrete(_Sigma):
    name = "KLMS"

    def __init__(self, steps, order=4, **kw):
        super().__init__(steps, **kw)
        self.order = order
        self.derivs = []
        # 16-point Gauss-Legendre on each interval (deterministic, no scipy)
        self._gl_x, self._gl_w = np.polynomial.legendre.leggauss(16)

    def _coef(self, order, t, cur):
        s = self.sigmas
        a, b = s[t], s[t + 1]
        xs = 0.5 * (b - a) * self._gl_x + 0.5 * (b + a)

        def basis(tau):
            prod = np.ones_like(tau)
            for k in range(order):
                if k == cur:
                    continue
                prod *= (tau - s[t - k]) / (s[t - cur] - s[t - k])
            return prod

        return float(0.5 * (b - a) * np.sum(self._gl_w * basis(xs)))

    def step(self, eps, i, x, generator=None):
        self.derivs.append(eps)  # d = (x - x0)/sigma = eps for eps-prediction
        if len(self.derivs) > self.order:
            self.derivs.pop(0)
        order = min(i + 1, self.order)
        coeffs = [self._coef(order, i, k) for k in range(order)]
        out = x
        for c, d in zip(coeffs, reversed(self.derivs)):
            out = out + c * d
        return out


class DPMSolverMultistep(Scheduler):
    """DPM-Solver++(2M), midpoint, lower-order-final (SD default config)."""
    name = "DPMSolverMultistep"

    def __init__(self, steps, **kw):
        super().__init__(steps, **kw)
        ts = np.linspace(0, self.n_train - 1, steps + 1).round()[::-1][:-1].astype(np.int64)
        self.timesteps = [int(v) for v in ts]
        self.prev_x0 = None
        self.prev_lambda = None

    def _coefs(self, t):
        if t < 0:
            return 1.0, 0.0, math.inf
        a = float(self.ac[t])
        alpha, sigma = math.sqrt(a), math.sqrt(1 - a)
        return alpha, sigma, math.log(alpha) - math.log(sigma)

    def step(self, eps, i, x, generator=None):
        t = self.timesteps[i]
        s = self.timesteps[i + 1] if i + 1 < len(self.timesteps) else -1
        a_t, s_t, l_t = self._coefs(t)
        a_s, s_s, l_s = self._coefs(s)
        x0 = (x - s_t * eps) / a_t
        last = i == len(self.timesteps) - 1
        lower_final = last and len(self.timesteps) < 15 or s < 0
        if s < 0:
            out = x0
        else:
            h = l_s - l_t
            em1 = math.expm1(-h)  # e^{-h} - 1
            out = (s_s / s_t) * x - a_s * em1 * x0
            if self.prev_x0 is not None and not lower_final:
                h0 = l_t - self.prev_lambda
                r0 = h0 / h
                d1 = (x0 - self.prev_x0) / r0
                out = out - 0.5 * a_s * em1 * d1
        self.prev_x0, self.prev_lambda = x0, l_t
        return out


class PNDM(Scheduler):
    """PLMS (PNDM with skip_prk_steps, SD default config)."""
    name = "PNDM"

    def __init__(self, steps, **kw):
        super().__init__(steps, **kw)
        base = self._leading(1)[::-1]  # ascending
        ts = np.array(base)
        plms = np.concatenate([ts[:-1], ts[-2:-1], ts[-1:]])[::-1]
        self.timesteps = [int(v) for v in plms]
        self.ratio = self.n_train // steps
        self.ets = []
        self.cur_sample = None
        self.counter = 0

    def _prev(self, x, t, tp, e):
        a_t = float(self.ac[t])
        a_p = float(self.ac[tp]) if tp >= 0 else float(self.ac[0])
        b_t, b_p = 1 - a_t, 1 - a_p
        coeff = (a_p / a_t) ** 0.5
        den = a_t * b_p ** 0.5 + (a_t * b_t * a_p) ** 0.5
        return coeff * x - (a_p - a_t) * e / den

    def step(self, eps, i, x, generator=None):
        t = self.timesteps[i]
        tp = t - self.ratio
        if self.counter != 1:
            self.ets = self.ets[-3:]
            self.ets.append(eps)
        else:
            tp = t
            t = t + self.ratio
        if len(self.ets) == 1 and self.counter == 0:
            e = eps
            self.cur_sample = x
        elif len(self.ets) == 1 and self.counter == 1:
            e = (eps + self.ets[-1]) / 2
            x = self.cur_sample
            self.cur_sample = None
        elif len(self.ets) == 2:
            e = (3 * self.ets[-1] - self.ets[-2]) / 2
        elif len(self.ets) == 3:
            e = (23 * self.ets[-1] - 16 * self.ets[-2] + 5 * self.ets[-3]) / 12
        else:
            e = (55 * self.ets[-1] - 59 * self.ets[-2] + 37 * self.ets[-3] - 9 * self.ets[-4]) / 24
        self.counter += 1
        return self._prev(x, t, tp, e)


def space_timesteps(n_train: int, steps: int) -> List[int]:
    """Evenly strided subset of the training timesteps (guided-diffusion
    ``space_timesteps(n, "K")`` with one section): round(i * (n-1)/(K-1))."""
    if steps == 1:
        return [0]
    stride = (n_train - 1) / (steps - 1)
    return sorted({int(round(i * stride)) for i in range(steps)})


class GaussianDiffusion(Scheduler):
    """Ancestral ``p_sample`` over a respaced DDPM (Kandinsky2 ``p_sampler``,
    ``docs/src/pages/register-model.mdx:140-168``).

    * ``predict``: "eps" (decoder UNet) or "x0" (diffusion prior);
    * ``learned_var``: the model's extra channels are the learned-range
      interpolation between log(beta_t) and the clipped posterior log-variance
      (improved-DDPM); otherwise the fixed-small posterior variance;
    * ``clamp``: pred_x0 clamp (Kandinsky decodes with clamp(-2, 2)).
    The respaced chain recomputes betas from the kept alphas_cumprod.
    ``step(out, i, x, generator, var=v)`` - ``v`` in [-1, 1] is the var head."""
    name = "p_sampler"
    needs_noise = True

    def __init__(self, steps, n_train=1000, schedule="linear", beta_start=0.0001, beta_end=0.02,
                 predict="eps", learned_var=True, clamp=None):
        full = sd_alphas_cumprod(n_train, beta_start, beta_end, schedule)
        use = space_timesteps(n_train, steps)
        ac = full[use]
        super().__init__(len(use), n_train, ac)
        ac_prev = np.concatenate([[1.0], ac[:-1]])
        self.betas = 1.0 - ac / ac_prev
        pv = self.betas * (1.0 - ac_prev) / (1.0 - ac)
        self.post_logvar = np.log(np.concatenate([[pv[1] if len(pv) > 1 else self.betas[0]], pv[1:]]))
        self.ac_prev = ac_prev
        self.use = use
        self.timesteps = [int(v) for v in use[::-1]]
        self.predict, self.learned_var, self.clamp = predict, learned_var, clamp

    def pred_x0(self, out, j, x):
        a = float(self.ac[j])
        if self.predict == "x0":
            x0 = out
        else:
            x0 = math.sqrt(1.0 / a) * x - math.sqrt(1.0 / a - 1.0) * out
        if self.clamp is not None:
            x0 = x0.clamp(-self.clamp, self.clamp)
        return x0

    def step(self, out, i, x, generator=None, var=None):
        j = len(self.use) - 1 - i              # respaced index, counting down
        a, ap, b = float(self.ac[j]), float(self.ac_prev[j]), float(self.betas[j])
        x0 = self.pred_x0(out.float(), j, x.float())
        mean = (b * math.sqrt(ap) / (1 - a)) * x0 + ((1 - ap) * math.sqrt(1 - b) / (1 - a)) * x.float()
        if j == 0:
            return mean
        if self.learned_var and var is not None:
            frac = (var.float() + 1.0) * 0.5
            logv = frac * math.log(b) + (1.0 - frac) * float(self.post_logvar[j])
            std = torch.exp(0.5 * logv)
        else:
            std = math.exp(0.5 * float(self.post_logvar[j]))
        return mean + std * _randn_like(x, generator)


SCHEDULERS = {
    "DDIM": DDIM,
    "K_EULER": EulerDiscrete,
    "K_EULER_ANCESTRAL": EulerAncestral,
    "DPMSolverMultistep": DPMSolverMultistep,
    "PNDM": PNDM,
    "KLMS": LMSDiscrete,
    "p_sampler": GaussianDiffusion,
}


def make_scheduler(name: str, steps: int) -> Scheduler:
    try:
        return SCHEDULERS[name](steps)
    except KeyError:
        raise ValueError(f"unknown scheduler {name!r}; choices {sorted(SCHEDULERS)}") from None
