"""SRRSModel (basicsr/models/srrs_model.py:16-88): the AMP train step of the remote-sensing configs.

``train.use_amp`` enables autocast; on MI355X the HIP kernels then run in bf16, which needs no
GradScaler (the reference uses fp16 + GradScaler, srrs_model.py:28-31, 79-82).  Like the
reference, a non-finite loss skips the optimizer step (srrs_model.py:65-77) — this check reads
the loss on the host, as the reference does.
"""
from collections import OrderedDict

import torch

from ..ops.conv import async_wgrad
from ..utils.registry import MODEL_REGISTRY
from .sr_model import SRModel


@MODEL_REGISTRY.register()
class SRRSModel(SRModel):

    def setup_optimizers(self):
        super().setup_optimizers()
        self.use_amp = bool(self.opt['train'].get('use_amp', False))
        self.amp_scaler = None  # bf16 autocast: no loss scaling

    def optimize_parameters(self, current_iter):
        self.optimizer_g.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=self.use_amp):
            self.output = self.net_g(self.lq)
        l_total = 0
        loss_dict = OrderedDict()
        if self.cri_pix:
            l_pix = self.cri_pix(self.output, self.gt)
            l_total += l_pix
            loss_dict['l_pix'] = l_pix
        self.log_dict = self.reduce_loss_dict(loss_dict)
        if not torch.isfinite(l_total).item():
            print('Loss is NaN or Inf. Skipping optimizer step.')
            self.log_nan_inf_loss(current_iter, l_total)
            self.optimizer_g.zero_grad()
            # drop this batch and its graph like the reference (srrs_model.py:68-77)
            del self.lq, self.gt, self.output
            return
        with async_wgrad(self.async_wgrad):
            l_total.backward()
        self.sync_gradients()
        if hasattr(self.optimizer_g, 'fp') and self.ema_decay > 0 and self.flat_ema is not None:
            self.optimizer_g.step(ema=self.flat_ema, ema_decay=self.ema_decay)
        else:
            self.optimizer_g.step()
            if self.ema_decay > 0:
                self.model_ema(decay=self.ema_decay)

    def log_nan_inf_loss(self, current_iter, loss):
        pass
