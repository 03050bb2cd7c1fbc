"""Diffusion samplers of the anythingv3 template's ``scheduler`` enum
(``templates/anythingv3.json:1``: DDIM, K_EULER, DPMSolverMultistep,
K_EULER_ANCESTRAL, PNDM, KLMS) plus the plain DDPM ancestral ``p_sampler``
used by Kandinsky2 (``docs/src/pages/register-model.mdx:140-168``).

Every sampler is expressed as ONE generic per-element update whose coefficients the host
computes per step (``StepPlan``)::

    e   = u + g (c - u)                                  classifier-free guidance
    E   = he0 e + he1 H[-1] + he2 H[-2] + he3 H[-3]      multistep history (PNDM, k-LMS)
    x0  = clamp(px X + pe E)                              eps- / x0-prediction
    out = ox Xsrc + oe E + ox0 x0 + od (x0 - P) + std N   (std learned: Kandinsky p_sample)

On a GPU the whole update of a lock-step group - CFG, sampler, the history / x0 stores and the
next step's bf16 UNet input - is ONE launch of ``ops/csrc/sampler.hip``; on CPU the same formula
runs in fp32 torch (``ops.ref.sampler_step``).  Ancestral noise is drawn from each task's CPU
generator up front, in exactly the order the step-by-step algorithm draws it, and copied to the
device once (no per-step host sync).  Formulas follow the published algorithms (DDIM,
Karras-Euler, DPM-Solver++(2M), PLMS, k-LMS, improved-DDPM p_sample); byte-parity with the
external Cog containers is "parity unpinned" (the reference ships no container outputs).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Tuple

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


@dataclass
class StepPlan:
    """Coefficients of one sampler step (see module docstring).  ``hist`` are offsets into the
    eps history (1 = the previous stored eps); ``store_hist`` appends this step's e."""
    he: Tuple[float, float, float, float] = (1.0, 0.0, 0.0, 0.0)
    hist: Tuple[int, int, int] = (1, 2, 3)
    store_hist: bool = False
    px: float = 0.0
    pe: float = 0.0
    clamp: Optional[float] = None
    ox: float = 0.0
    oe: float = 0.0
    ox0: float = 0.0
    od: float = 0.0
    std: float = 0.0
    learned: Optional[Tuple[float, float]] = None     # (log beta, posterior log var) of p_sample
    noise: bool = False
    store_x0: bool = False
    read_p: bool = False
    use_cur: bool = False
    store_cur: bool = False
    in_scale: float = 1.0                             # scale_model_input of THIS step


class Scheduler:
    name = "base"
    init_noise_sigma = 1.0

    def __init__(self, steps: int, n_train: int = 1000, alphas_cumprod=None):
        self.steps = steps
        self.n_train = n_train
        self.ac = sd_alphas_cumprod(n_train) if alphas_cumprod is None else np.asarray(alphas_cumprod)
        self.timesteps: List[float] = []

    def in_scale(self, i) -> float:
        return 1.0

    def plans(self) -> List[StepPlan]:
        """All steps' plans, in order (schedulers with multistep state advance it here)."""
        out = []
        for i in range(len(self.timesteps)):
            p = self._plan(i)
            p.in_scale = self.in_scale(i)
            out.append(p)
        return out

    def _plan(self, i) -> StepPlan:
        raise NotImplementedError

    def _leading(self, offset=1):
        ratio = self.n_train // self.steps
        return [int(v) for v in (np.arange(0, self.steps) * ratio).round()[::-1] + offset]


def ldm_uniform_timesteps(n_train: int, steps: int) -> List[int]:
    """latent-diffusion ``make_ddim_timesteps("uniform")``: range(0, n_train, n_train // steps) + 1,
    ascending (more than ``steps`` entries when ``steps`` does not divide ``n_train``, as there)."""
    c = max(1, n_train // steps)
    ts = [t + 1 for t in range(0, n_train, c)]
    if ts[-1] >= n_train:
        raise ValueError(f"{steps} steps over {n_train} training steps: timestep {ts[-1]} out of range")
    return ts


class DDIM(Scheduler):
    """DDIM (eta 0 by default).  ``timesteps_asc``: an explicit ascending timestep list (the
    latent-diffusion uniform discretisation of the Kandinsky 2 ``ddim_sampler``); the previous
    alpha of the first (smallest) timestep is alphas_cumprod[0] in both conventions."""
    name = "DDIM"

    def __init__(self, steps, eta=0.0, timesteps_asc: Optional[List[int]] = None, **kw):
        super().__init__(steps, **kw)
        self.eta = eta
        self.timesteps = list(timesteps_asc[::-1]) if timesteps_asc is not None else self._leading(1)
        self.ratio = self.n_train // steps

    def _plan(self, i):
        t = self.timesteps[i]
        tp = self.timesteps[i + 1] if i + 1 < len(self.timesteps) else -1
        a_t = float(self.ac[t])
        a_p = float(self.ac[tp]) if tp >= 0 else float(self.ac[0])
        var = (1 - a_p) / (1 - a_t) * (1 - a_t / a_p)
        std = self.eta * math.sqrt(max(var, 0.0))
        return StepPlan(px=1.0 / math.sqrt(a_t), pe=-math.sqrt(1 - a_t) / math.sqrt(a_t), ox0=math.sqrt(a_p),
                        oe=math.sqrt(max(1 - a_p - std * std, 0.0)), std=std, noise=std > 0)


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

    def in_scale(self, i):
        return 1.0 / math.sqrt(self.sigmas[i] ** 2 + 1)


class EulerDiscrete(_Sigma):
    name = "K_EULER"

    def _plan(self, i):
        s, sn = self.sigmas[i], self.sigmas[i + 1]
        return StepPlan(ox=1.0, oe=float(sn - s))


class EulerAncestral(_Sigma):
    name = "K_EULER_ANCESTRAL"

    def _plan(self, i):
        s, sn = self.sigmas[i], self.sigmas[i + 1]
        up = math.sqrt(max(sn ** 2 * (s ** 2 - sn ** 2) / s ** 2, 0.0))
        down = math.sqrt(max(sn ** 2 - up ** 2, 0.0))
        return StepPlan(ox=1.0, oe=float(down - s), std=up, noise=up > 0)


class LMSDiscrete(_Sigma):
    name = "KLMS"

    def __init__(self, steps, order=4, **kw):
        super().__init__(steps, **kw)
        self.order = order
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

    def _plan(self, i):
        # d = (x - x0) / sigma = eps for eps-prediction; the last `order` d's, newest first
        order = min(i + 1, self.order)
        c = [self._coef(order, i, k) for k in range(order)] + [0.0] * (4 - order)
        return StepPlan(he=tuple(c), store_hist=True, ox=1.0, oe=1.0)


class DPMSolverMultistep(Scheduler):
    """DPM-Solver++(2M), midpoint, lower-order-final (SD default config)."""
    name = "DPMSolverMultistep"

    def __init__(self, steps, **kw):
        super().__init__(steps, **kw)
        ts = np.linspace(0, self.n_train - 1, steps + 1).round()[::-1][:-1].astype(np.int64)
        self.timesteps = [int(v) for v in ts]

    def _coefs(self, t):
        if t < 0:
            return 1.0, 0.0, math.inf
        a = float(self.ac[t])
        alpha, sigma = math.sqrt(a), math.sqrt(1 - a)
        return alpha, sigma, math.log(alpha) - math.log(sigma)

    def plans(self):
        out, prev_lambda = [], None
        n = len(self.timesteps)
        for i, t in enumerate(self.timesteps):
            s = self.timesteps[i + 1] if i + 1 < n else -1
            a_t, s_t, l_t = self._coefs(t)
            a_s, s_s, l_s = self._coefs(s)
            p = StepPlan(px=1.0 / a_t, pe=-s_t / a_t, store_x0=True)
            lower_final = (i == n - 1) and n < 15 or s < 0
            if s < 0:
                p.ox0 = 1.0
            else:
                h = l_s - l_t
                em1 = math.expm1(-h)                       # e^{-h} - 1
                p.ox, p.ox0 = s_s / s_t, -a_s * em1
                if prev_lambda is not None and not lower_final:
                    r0 = (l_t - prev_lambda) / h
                    p.od, p.read_p = -0.5 * a_s * em1 / r0, True
            prev_lambda = l_t
            out.append(p)
        return out


class PNDM(Scheduler):
    """PLMS (PNDM with skip_prk_steps, SD default config).  Also the latent-diffusion PLMSSampler of
    the Kandinsky 2 ``plms_sampler``: its first step (e_t, a DDIM probe to t_next, e = (e_t +
    e_t_next) / 2 from the original x) and the 2/3/4-step Adams-Bashforth weights are this
    schedule's counter-0/1 pair and ets history, and its DDIM update equals PNDM's formula (eq. 9)
    algebraically.  ``timesteps_asc``: an explicit uniform ascending list (stride = ratio)."""
    name = "PNDM"

    def __init__(self, steps, timesteps_asc: Optional[List[int]] = None, **kw):
        super().__init__(steps, **kw)
        base = list(timesteps_asc) if timesteps_asc is not None else self._leading(1)[::-1]  # ascending
        ts = np.array(base)
        plms = np.concatenate([ts[:-1], ts[-2:-1], ts[-1:]])[::-1]
        self.timesteps = [int(v) for v in plms]
        self.ratio = int(ts[1] - ts[0]) if len(ts) > 1 else self.n_train // steps

    def _prev_coefs(self, t, tp):
        a_t = float(self.ac[t])
        a_p = float(self.ac[tp]) if tp >= 0 else float(self.ac[0])
        b_t, b_p = 1 - a_t, 1 - a_p
        den = a_t * b_p ** 0.5 + (a_t * b_t * a_p) ** 0.5
        return (a_p / a_t) ** 0.5, -(a_p - a_t) / den

    def plans(self):
        out, n_ets = [], 0
        for counter, t in enumerate(self.timesteps):
            tp = t - self.ratio
            p = StepPlan()
            if counter != 1:
                n_ets = min(n_ets + 1, 4)
                p.store_hist = True
            else:
                tp, t = t, t + self.ratio
            if n_ets == 1 and counter == 0:
                p.he, p.store_cur = (1.0, 0.0, 0.0, 0.0), True
            elif n_ets == 1 and counter == 1:
                p.he, p.use_cur = (0.5, 0.5, 0.0, 0.0), True          # (eps + ets[-1]) / 2 on the stored x
            elif n_ets == 2:
                p.he = (1.5, -0.5, 0.0, 0.0)
            elif n_ets == 3:
                p.he = (23 / 12, -16 / 12, 5 / 12, 0.0)
            else:
                p.he = (55 / 24, -59 / 24, 37 / 24, -9 / 24)
            p.ox, p.oe = self._prev_coefs(t, tp)
            out.append(p)
        return out


def space_timesteps(n_train: int, spec) -> List[int]:
    """guided-diffusion ``space_timesteps`` (the respacing of Kandinsky 2's ``p_sampler`` and of its
    prior's ``prior_steps`` string): an int / "K" (one section), "K1,K2,..." (equal sections, the
    first ``n % len`` one step longer, each strided by accumulating (size-1)/(K-1) and rounding),
    or "ddimK" (the stride i with len(range(0, n, i)) == K)."""
    if isinstance(spec, str) and spec.startswith("ddim"):
        want = int(spec[len("ddim"):])
        for i in range(1, n_train):
            if len(range(0, n_train, i)) == want:
                return list(range(0, n_train, i))
        raise ValueError(f"cannot create exactly {want} steps with an integer stride")
    counts = [int(x) for x in str(spec).split(",")] if isinstance(spec, str) else [int(spec)]
    if not counts or any(c < 1 for c in counts):
        raise ValueError(f"bad respacing {spec!r}")
    size_per, extra = divmod(n_train, len(counts))
    start, out = 0, []
    for i, count in enumerate(counts):
        size = size_per + (1 if i < extra else 0)
        if size < count:
            raise ValueError(f"cannot divide a section of {size} steps into {count}")
        frac = 1.0 if count <= 1 else (size - 1) / (count - 1)
        cur = 0.0
        for _ in range(count):
            out.append(start + round(cur))
            cur += frac
        start += size
    return sorted(set(out))


class GaussianDiffusion(Scheduler):
    """Ancestral ``p_sample`` over a respaced DDPM (Kandinsky2 ``p_sampler``,
    ``docs/src/pages/register-model.mdx:140-168``).

    * ``predict``: "eps" (decoder UNet) or "x0" (diffusion prior);
    * ``learned_var``: the model's extra channels are the learned-range
      interpolation between log(beta_t) and the clipped posterior log-variance
      (improved-DDPM); otherwise the fixed-small posterior variance;
    * ``clamp``: pred_x0 clamp (Kandinsky decodes with clamp(-2, 2)).
    The respaced chain recomputes betas from the kept alphas_cumprod."""
    name = "p_sampler"

    def __init__(self, steps, n_train=1000, schedule="linear", beta_start=0.0001, beta_end=0.02,
                 predict="eps", learned_var=True, clamp=None):
        full = sd_alphas_cumprod(n_train, beta_start, beta_end, schedule)
        use = space_timesteps(n_train, steps)    # int, "K", "K1,K2", "ddimK"
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

    def _plan(self, i):
        j = len(self.use) - 1 - i              # respaced index, counting down
        a, ap, b = float(self.ac[j]), float(self.ac_prev[j]), float(self.betas[j])
        p = StepPlan(clamp=self.clamp, ox0=b * math.sqrt(ap) / (1 - a), ox=(1 - ap) * math.sqrt(1 - b) / (1 - a))
        if self.predict == "x0":
            p.px, p.pe = 0.0, 1.0
        else:
            p.px, p.pe = math.sqrt(1.0 / a), -math.sqrt(1.0 / a - 1.0)
        if j > 0:
            p.noise = True
            if self.learned_var:
                p.learned = (math.log(b), float(self.post_logvar[j]))
            else:
                p.std = math.exp(0.5 * float(self.post_logvar[j]))
        return p


SCHEDULERS = {
    "DDIM": DDIM,
    "K_EULER": EulerDiscrete,
    "K_EULER_ANCESTRAL": EulerAncestral,
    "DPMSolverMultistep": DPMSolverMultistep,
    "PNDM": PNDM,
    "KLMS": LMSDiscrete,
    "p_sampler": GaussianDiffusion,
}


# Kandinsky 2 template ``scheduler`` enum (docs/src/pages/register-model.mdx:141-185):
# p_sampler = respaced ancestral p_sample (learned variance, clamp); ddim_sampler / plms_sampler =
# the latent-diffusion samplers over the FULL 1000-step linear schedule with uniform timesteps,
# eps = the UNet's first 4 channels, no clamp.  The template lists "pims_sampler": taken as PLMS.
K2_SCHEDULERS = ("p_sampler", "ddim_sampler", "pims_sampler", "plms_sampler")


def k2_decoder_scheduler(name: str, steps: int, clamp: float = 2.0) -> Scheduler:
    if name == "p_sampler":
        return GaussianDiffusion(steps, schedule="linear", predict="eps", learned_var=True, clamp=clamp)
    ac = sd_alphas_cumprod(1000, 0.0001, 0.02, "linear")
    ts = ldm_uniform_timesteps(1000, steps)
    if name == "ddim_sampler":
        return DDIM(steps, timesteps_asc=ts, alphas_cumprod=ac)
    if name in ("pims_sampler", "plms_sampler"):
        return PNDM(steps, timesteps_asc=ts, alphas_cumprod=ac)
    raise ValueError(f"unknown Kandinsky 2 scheduler {name!r}; choices {K2_SCHEDULERS}")


def make_scheduler(name: str, steps: int) -> Scheduler:
    try:
        return SCHEDULERS[name](steps)
    except KeyError:
        raise ValueError(f"unknown scheduler {name!r}; choices {sorted(SCHEDULERS)}") from None


# ---------------------------------------------------------------------------------------------
class TaskSampler:
    """One task's sampler state on the device: fp32 latent X, previous x0 P, PNDM's stored
    sample, a 4-slot eps history ring, and the task's whole ancestral-noise sequence (drawn now
    from its CPU generator in step order, copied once with a non-blocking H2D from pinned memory)."""

    def __init__(self, sched: Scheduler, x: torch.Tensor, gen: Optional[torch.Generator], device,
                 plans: Optional[List[StepPlan]] = None):
        self.sched = sched
        self.plans = plans if plans is not None else sched.plans()
        dev = torch.device(device)
        self.x = x.detach().to(device=dev, dtype=torch.float32, copy=True).contiguous()   # never alias the caller
        shape = self.x.shape
        need = lambda f: any(f(p) for p in self.plans)             # noqa: E731
        self.p = torch.zeros(shape, dtype=torch.float32, device=dev) if need(lambda p: p.store_x0 or p.read_p) \
            else None
        self.cur = torch.zeros(shape, dtype=torch.float32, device=dev) if need(lambda p: p.store_cur) else None
        self.hist = torch.zeros((4,) + tuple(shape), dtype=torch.float32, device=dev) if need(
            lambda p: p.store_hist) else None
        self.n_hist = 0
        self.noise_idx = []
        k = 0
        for p in self.plans:
            self.noise_idx.append(k if p.noise else -1)
            k += int(p.noise)
        self.noise = None
        if k:
            if gen is None:
                raise ValueError("an ancestral sampler needs the task's generator")
            draws = torch.stack([torch.randn(tuple(shape), generator=gen, dtype=torch.float32) for _ in range(k)])
            if dev.type == "cuda":
                draws = draws.pin_memory()
            self.noise = draws.to(dev, non_blocking=True)

    def hist_slot(self, back: int) -> Optional[torch.Tensor]:
        """The eps stored ``back`` appends ago (1 = most recent), or None."""
        if self.hist is None or back > self.n_hist or back > 4:
            return None
        return self.hist[(self.n_hist - back) % 4]

    def task_args(self, i: int, u, c, g: float, xin0=None, xin1=None, next_scale: float = 1.0) -> dict:
        p = self.plans[i]
        h = [self.hist_slot(b) if coef != 0.0 else None for b, coef in zip(p.hist, p.he[1:])]
        return {"u": u, "c": c, "x": self.x, "xsrc": self.cur if p.use_cur else self.x, "p": self.p,
                "cur": self.cur, "hs": self.hist[self.n_hist % 4] if p.store_hist else None,
                "h1": h[0], "h2": h[1], "h3": h[2],
                "noise": self.noise[self.noise_idx[i]] if p.noise else None, "xin0": xin0, "xin1": xin1,
                "g": g, "he": p.he, "px": p.px, "pe": p.pe, "clamp": p.clamp, "ox": p.ox, "oe": p.oe,
                "ox0": p.ox0, "od": p.od, "std": p.std, "learned": p.learned, "in_scale": next_scale,
                "store_x0": p.store_x0, "store_cur": p.store_cur, "read_p": p.read_p}

    def advance(self, i: int):
        if self.plans[i].store_hist:
            self.n_hist += 1


class GroupSampler:
    """The k tasks of one lock-step group (k = 1 for a solo task): ``step(i, out)`` runs the fused
    CFG + sampler update of every task from the UNet output ``out`` and writes the next step's
    UNet input into ``xin`` (one HIP launch on a GPU).

    ``rows(k)`` -> (uncond view, cond view, xin view 0, xin view 1) of task k."""

    def __init__(self, tasks: List[TaskSampler], guidance: List[float], xin: torch.Tensor, rows):
        self.tasks, self.g, self.xin, self.rows = tasks, guidance, xin, rows
        self.n = len(tasks[0].plans)

    def write_input(self, i: int = 0):
        """xin <- bf16(X * in_scale(i)) for every task (once, before the first UNet call)."""
        for k, t in enumerate(self.tasks):
            _, _, d0, d1 = self.rows(k, None)
            v = (t.x * t.plans[i].in_scale).to(self.xin.dtype)
            d0.copy_(v.reshape(d0.shape))
            if d1 is not None:
                d1.copy_(v.reshape(d1.shape))

    def step(self, i: int, out: torch.Tensor):
        from .. import ops
        last = i == self.n - 1
        args = []
        for k, t in enumerate(self.tasks):
            u, c, d0, d1 = self.rows(k, out)
            nscale = 1.0 if last else t.plans[i + 1].in_scale
            args.append(t.task_args(i, u, c, self.g[k], None if last else d0, None if last else d1, nscale))
        ops.sampler_step(args)
        for t in self.tasks:
            t.advance(i)

    def latent(self, k: int) -> torch.Tensor:
        return self.tasks[k].x
