"""Dynamic loss scaling for fp16 training, decided on the device.

Reference: the DDP / FSDP path of train_harness.py runs fp16 autocast with
``torch.cuda.amp.GradScaler()`` (train_harness.py:334-335, 371-376): the loss is multiplied by a
scale S before backward, the optimizer step is skipped when any gradient is inf / nan, and S
halves on such a step and doubles after 2000 clean ones.  torch's scaler reads ``found_inf`` on the
host (``.item()``, torch/amp/grad_scaler.py); here the whole decision stays on the GPU:

* ``state`` = f32[4] on the device: [S, growth tracker, optimizer steps taken, steps skipped];
* backward seeds the autograd graph with S itself (``loss.backward(scaler.grad_output)``), so the
  fp16 gradients are S-scaled with no extra pass;
* at the optimizer step the engine's gradient-norm pass (``sumsq``, all-reduced where sharded) is
  the inf check: a non-finite sum means an inf / nan gradient.  ``amp_step`` (csrc/adamw.hip) then
  sets the AdamW skip flag (hp[3]) or the unscale + clip coefficient and the bias corrections of
  the device step count, and updates S -- one 1-thread kernel, no host sync, HIP-graph safe.

On the CPU the same arithmetic runs in torch (the engines' CPU path trains in fp32, where the
scaler only exercises the bookkeeping).
"""
import math

import torch

from ..ops._ext import ext


class DynamicLossScaler:
    def __init__(self, device, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000):
        self.device = torch.device(device)
        self.growth, self.backoff, self.interval = float(growth_factor), float(backoff_factor), int(growth_interval)
        self.state = torch.tensor([float(init_scale), 0.0, 0.0, 0.0], dtype=torch.float32, device=self.device)
        self.last_skipped = False        # CPU path only (the GPU path never syncs)

    @property
    def grad_output(self) -> torch.Tensor:
        """The backward seed: d(loss) = S (0-dim view of the device state)."""
        return self.state[0]

    def scale(self) -> float:
        return float(self.state[0].item())

    def stats(self) -> dict:
        s = self.state.tolist()
        return {"loss_scale": s[0], "growth_tracker": int(s[1]), "optimizer_steps_taken": int(s[2]),
                "optimizer_steps_skipped": int(s[3])}

    def step(self, norm_sq: torch.Tensor, coef: torch.Tensor, norm_out, hp, max_norm: float,
             extra_scale: float, betas):
        """Decide skip / unscale for one optimizer step (see the module docstring)."""
        b1, b2 = betas
        if norm_sq.is_cuda:
            ext().amp_step(norm_sq, self.state, coef, norm_out, hp, float(max_norm), float(extra_scale),
                           float(b1), float(b2), self.growth, self.backoff, self.interval)
            return
        S = float(self.state[0])
        nsq = float(norm_sq[0])
        if not math.isfinite(nsq):
            self.state[0] = S * self.backoff
            self.state[1] = 0.0
            self.state[3] += 1.0
            coef.fill_(0.0)
            self.last_skipped = True
            if norm_out is not None:
                norm_out.fill_(nsq)
            return
        nrm = math.sqrt(nsq) / S * extra_scale
        c = min(1.0, max_norm / (nrm + 1e-6)) if max_norm > 0 else 1.0
        coef.fill_(c * extra_scale / S)
        if norm_out is not None:
            norm_out.fill_(nrm)
        self.state[2] += 1.0
        tr = float(self.state[1]) + 1.0
        if tr >= self.interval:
            self.state[0] = S * self.growth
            tr = 0.0
        self.state[1] = tr
        self.last_skipped = False

    def state_dict(self):
        return {"state": self.state.detach().cpu().clone(), "growth": self.growth, "backoff": self.backoff,
                "interval": self.interval}

    def load_state_dict(self, sd):
        self.state.copy_(sd["state"])
