"""SwinIRModel (basicsr/models/swinir_model.py:11-36): reflect-pad the LR input to a multiple
of window_size for inference, crop the output by pad * scale.  (The padding of the NCHW input
uses torch's device pad — validation-only, not the train hot path.)"""
import torch
from torch.nn import functional as F

from ..utils.registry import MODEL_REGISTRY
from .sr_model import SRModel
from .srrs_model import SRRSModel


@MODEL_REGISTRY.register()
class SwinIRModel(SRModel):

    def test(self):
        window_size = self.opt['network_g']['window_size']
        scale = self.opt.get('scale', 1)
        _, _, h, w = self.lq.size()
        mod_pad_h = (window_size - h % window_size) % window_size
        mod_pad_w = (window_size - w % window_size) % window_size
        img = F.pad(self.lq, (0, mod_pad_w, 0, mod_pad_h), 'reflect')
        net = self.net_g_ema if hasattr(self, 'net_g_ema') else self.net_g
        was_training = self.net_g.training
        net.eval()
        with torch.no_grad():
            self.output = net(img)
        if net is self.net_g and was_training:
            self.net_g.train()
        _, _, h, w = self.output.size()
        self.output = self.output[:, :, 0:h - mod_pad_h * scale, 0:w - mod_pad_w * scale]


@MODEL_REGISTRY.register()
class SwinIRRSModel(SwinIRModel, SRRSModel):
    pass
