"""SRRSModel (basicsr/models/srrs_model.py:16-251): the AMP train step and the [-1, 1] validation of
the fork's remote-sensing configs.

``train.use_amp`` enables autocast; on MI355X the HIP kernels then run in bf16, which needs no
GradScaler (the reference uses fp16 + GradScaler, srrs_model.py:28-31, 79-82).  Like the
reference, a non-finite loss skips the optimizer step (srrs_model.py:65-77) — this check reads
the loss on the host, as the reference does.

Validation (srrs_model.py:93-138) works on tensors in [-1, 1]: every visual goes through
``minusone_one_tensor_to_ubyte_numpy`` (clamp, (x + 1) / 2, make_grid, img_as_ubyte; channel
order kept), the metrics compare the ``sr`` and ``gt`` images, each image's scores go into a
per-image table written as ``<visualization>/<dataset>_<iter>.csv`` (srrs_model.py:214-216), and
saved visuals are split into RGB (channels 0-2) and NIR (channel 3) PNGs (srrs_model.py:194-212).
"""
import os
from collections import OrderedDict
from os import path as osp

import pandas as pd
import torch

from ..metrics import calculate_metric
from ..ops.conv import async_wgrad
from ..utils.img_util import imwrite, minusone_one_tensor_to_ubyte_numpy
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
        try:
            with async_wgrad(self.async_wgrad, blocks=getattr(self, 'async_blocks', None)):
                l_total.backward()
        except BaseException:
            # a failed backward leaves the DDP reducer mid-step (buckets issued, counts short):
            # join and reset it so a caller that skips the batch can keep training
            red = getattr(self.net_g, 'reducer', None)
            if red is not None:
                red.abandon_step()
            raise
        self.sync_gradients()
        if hasattr(self.optimizer_g, 'fp') and self.ema_decay > 0 and self.flat_ema is not None:
            self.optimizer_g.step(ema=self.flat_ema, ema_decay=self.ema_decay)
        else:
            self.optimizer_g.step()
            if self.ema_decay > 0:
                self.model_ema(decay=self.ema_decay)

    def log_nan_inf_loss(self, current_iter, loss):
        pass

    # ---- validation on [-1, 1] tensors ------------------------------------------------------
    def get_current_visuals(self, current_iter=None):
        """The fork's visual keys (basicsr/models/sr_model.py:265-272): ``lq``, ``sr`` and its
        per-iteration copy ``sr_<iter>``, ``gt``."""
        out = OrderedDict()
        out['lq'] = self.lq.detach().float().cpu()
        out['sr'] = self.output.detach().float().cpu()
        out[f'sr_{current_iter}'] = out['sr']
        if hasattr(self, 'gt'):
            out['gt'] = self.gt.detach().float().cpu()
        return out

    def nondist_validation(self, dataloader, current_iter, tb_logger, save_img):
        dataset_name = dataloader.dataset.opt['name']
        metrics_enabled = self.opt['val'].get('metrics') is not None
        if metrics_enabled:
            self._prepare_metrics(dataset_name)
        detailed = pd.DataFrame()  # one row per image, one column per metric (srrs_model.py:101)
        idx = -1
        for idx, val_data in enumerate(dataloader):
            img_name = self._extract_img_name(val_data)
            self.feed_data(val_data)
            self.test()
            visuals = self.get_current_visuals(current_iter)
            converted = {k: minusone_one_tensor_to_ubyte_numpy(v) for k, v in visuals.items() if v is not None}
            self._release_gpu_memory()
            if metrics_enabled and 'sr' in converted and 'gt' in converted:
                self._compute_metrics(img_name, converted['sr'], converted['gt'], detailed)
                converted.pop('sr')  # evaluated only, not saved
            if save_img:
                self._save_visuals(dataset_name, img_name, converted)
        if metrics_enabled:
            self._finalize_metrics(idx + 1, dataset_name, current_iter, tb_logger)
            self._save_metrics_csv(dataset_name, current_iter, detailed)

    def _prepare_metrics(self, dataset_name):
        if not hasattr(self, 'metric_results'):
            self.metric_results = {name: 0.0 for name in self.opt['val']['metrics']}
        self._initialize_best_metric_results(dataset_name)
        self.metric_results = {metric: 0 for metric in self.metric_results}

    @staticmethod
    def _extract_img_name(val_data):
        """srrs_model.py:150-152: a TACO sample's name is the basename of its first path; any other
        path keeps its directories, without the extension."""
        lq_path = val_data['lq_path'][0]
        return osp.basename(lq_path.split(',')[0]) if lq_path.endswith('.taco') else osp.splitext(lq_path)[0]

    def _release_gpu_memory(self):
        for attr in ('lq', 'output', 'gt'):
            if hasattr(self, attr):
                delattr(self, attr)

    def _compute_metrics(self, img_name, sr_img, gt_img, detailed):
        if gt_img is None:
            return
        data = {'img': sr_img, 'img2': gt_img}
        scores = {name: calculate_metric(data, opt_) for name, opt_ in self.opt['val']['metrics'].items()}
        for name, score in scores.items():
            detailed.loc[img_name, name] = score
            self.metric_results[name] += score

    def _finalize_metrics(self, total, dataset, iter_num, tb_logger):
        for name in self.metric_results:
            self.metric_results[name] /= total
            self._update_best_metric_result(dataset, name, self.metric_results[name], iter_num)
        self._log_validation_metric_values(iter_num, dataset, tb_logger)

    def _save_metrics_csv(self, dataset, iter_num, detailed):
        """``<visualization>/<dataset>_<iter>.csv``, the per-image table (srrs_model.py:214-216)."""
        vis = self.opt['path']['visualization']
        os.makedirs(vis, exist_ok=True)
        detailed.to_csv(osp.join(vis, f'{dataset}_{iter_num}.csv'))

    def _save_visuals(self, dataset, img_name, images):
        """RGB (channels 0-2) and NIR (channel 3) PNGs of every visual, each written once
        (srrs_model.py:194-212, 218-232).  Deviation: an absolute image name (a non-TACO path) is
        reduced to its basename, where the reference's ``osp.join`` would leave the visualization
        directory; a visual without a fourth channel has no NIR file (the reference raises)."""
        vis = self.opt['path']['visualization']
        if osp.isabs(img_name):
            img_name = osp.basename(img_name)
        for key, img in images.items():
            if img is None:
                continue
            rgb = osp.join(vis, 'RGB', dataset, img_name, f'{key}.png')
            if not osp.exists(rgb):
                imwrite(img[..., :3][..., ::-1], rgb)  # imwrite takes BGR (cv2 convention)
            if img.shape[-1] > 3:
                nir = osp.join(vis, 'NIR', dataset, img_name, f'{key}.png')
                if not osp.exists(nir):
                    imwrite(img[..., 3], nir)
