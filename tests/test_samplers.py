"""The generic fused-sampler form (StepPlan coefficients + ops.ref.sampler_step, the fp32 twin of
ops/csrc/sampler.hip) reproduces every textbook sampler step by step: DDIM (eta 0 and 1),
Euler, Euler-ancestral, DPM-Solver++(2M), PNDM/PLMS, k-LMS and p_sample (eps / x0 prediction,
learned variance, clamp), including the order in which ancestral noise is drawn from the task's
generator and classifier-free guidance on separate uncond / cond rows."""

import pytest
import torch

from arbius_amd.models import schedulers as S
from oracles import step_samplers as O

SHAPE = (1, 6, 5, 4)


def _run_new(sched, x, seed, eps_seq, var_seq, g):
    gen = torch.Generator().manual_seed(seed)
    ts = S.TaskSampler(sched, x, gen, "cpu")
    xin = torch.empty((2,) + SHAPE[1:])
    cout = 8 if var_seq is not None else 4

    def rows(k, out):
        return (None if out is None else out[0], None if out is None else out[1], xin[0], xin[1])

    samp = S.GroupSampler([ts], [g], xin, rows)
    samp.write_input(0)
    for i in range(len(ts.plans)):
        assert torch.allclose(xin[0], (ts.x * ts.plans[i].in_scale)[0], rtol=1e-6, atol=1e-6)
        u, c = eps_seq[i]
        if cout == 8:
            u = torch.cat([u, var_seq[i]], -1)
            c = torch.cat([c, var_seq[i]], -1)
        samp.step(i, torch.cat([u, c]))
    return ts.x


def _run_old(sched, x, seed, eps_seq, var_seq, g):
    gen = torch.Generator().manual_seed(seed)
    x = x.clone()
    for i in range(len(sched.timesteps)):
        u, c = eps_seq[i]
        e = u + g * (c - u)
        if var_seq is not None:
            x = sched.step(e, i, x, gen, var=var_seq[i])
        else:
            x = sched.step(e, i, x, gen)
    return x


CASES = [
    ("DDIM", lambda: (S.DDIM(7), O.DDIM(7))),
    ("DDIM-eta1", lambda: (S.DDIM(7, eta=1.0), O.DDIM(7, eta=1.0))),
    ("K_EULER", lambda: (S.EulerDiscrete(7), O.EulerDiscrete(7))),
    ("K_EULER_ANCESTRAL", lambda: (S.EulerAncestral(7), O.EulerAncestral(7))),
    ("DPMSolverMultistep", lambda: (S.DPMSolverMultistep(9), O.DPMSolverMultistep(9))),
    ("DPMSolverMultistep-20", lambda: (S.DPMSolverMultistep(20), O.DPMSolverMultistep(20))),
    ("PNDM", lambda: (S.PNDM(8), O.PNDM(8))),
    ("KLMS", lambda: (S.LMSDiscrete(8), O.LMSDiscrete(8))),
    ("p_sampler-eps-learned", lambda: (S.GaussianDiffusion(6, clamp=2.0), O.GaussianDiffusion(6, clamp=2.0))),
    ("p_sampler-x0-prior", lambda: (S.GaussianDiffusion(5, schedule="cosine", predict="x0", learned_var=False),
                                    O.GaussianDiffusion(5, schedule="cosine", predict="x0", learned_var=False))),
]


@pytest.mark.parametrize("name,make", CASES, ids=[c[0] for c in CASES])
def test_generic_sampler_matches_textbook(name, make):
    new, old = make()
    n = len(old.timesteps)
    assert new.timesteps == old.timesteps and new.init_noise_sigma == old.init_noise_sigma
    g = torch.Generator().manual_seed(5)
    x = torch.randn(SHAPE, generator=g) * old.init_noise_sigma
    eps = [(torch.randn(SHAPE, generator=g), torch.randn(SHAPE, generator=g)) for _ in range(n)]
    learned = isinstance(old, O.GaussianDiffusion) and old.learned_var
    var = [torch.rand(SHAPE, generator=g) * 2 - 1 for _ in range(n)] if learned else None
    # the textbook loop feeds scale_model_input(x) to the model; the generic form writes it into xin
    a = _run_new(new, x, 1234, eps, var, 7.5)
    b = _run_old(old, x, 1234, eps, var, 7.5)
    scale = max(1.0, b.abs().max().item())
    assert torch.allclose(a, b, rtol=1e-4, atol=1e-4 * scale), (name, (a - b).abs().max().item())


def test_noise_is_predrawn_in_step_order():
    sched = S.EulerAncestral(6)
    gen = torch.Generator().manual_seed(9)
    x = torch.zeros(SHAPE)
    ts = S.TaskSampler(sched, x, gen, "cpu")
    ref = torch.Generator().manual_seed(9)
    want = [torch.randn(SHAPE, generator=ref) for p in ts.plans if p.noise]
    assert ts.noise.shape[0] == len(want) == 5          # the last step (sigma 0) draws nothing
    for a, b in zip(ts.noise, want):
        assert torch.equal(a, b)
