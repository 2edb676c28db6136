"""Single-image SR model (mirror of basicsr/models/sr_model.py:16-279 and the AMP variant
basicsr/models/srrs_model.py:33-88).

The train step ``optimize_parameters`` is the north-star hot path: zero_grad -> net_g
forward on the HIP engine -> L1 (fused HIP reduction + gradient) -> backward (HIP conv
dgrad/wgrad; bucketed RCCL all-reduce launched from backward hooks when distributed) ->
one fused Adam + EMA kernel over the flat parameter vector.  No host synchronisation
inside the step (the loss log is reduced when read).

AMP: ``train.use_amp`` (SRRSModel's key) turns on autocast; the HIP kernels then compute
in bf16 (the reference uses fp16 + GradScaler; bf16 needs no loss scaling).
"""
from collections import OrderedDict
from os import path as osp

import torch

from ..archs import build_network
from ..losses import build_loss
from ..metrics import calculate_metric

from ..ops.conv import async_wgrad, bump_param_epoch, take_captured_tables
from ..utils.flat import FlatParams
from ..utils.img_util import imwrite, tensor2img
from ..utils.logger import get_root_logger
from ..utils.registry import MODEL_REGISTRY
from ..utils.step_graph import SegmentedStepGraph
from .base_model import BaseModel, SRDistributed
from .._switches import switch


@MODEL_REGISTRY.register()
class SRModel(BaseModel):

    def build_optional_loss(self, opt_dict, key):
        if key not in opt_dict or opt_dict[key] is None:
            return None
        if key == 'perceptual_opt':
            raise NotImplementedError('PerceptualLoss needs pretrained VGG weights; out of scope (SURVEY.md §2a)')
        return build_loss(opt_dict[key]).to(self.device)

    def __init__(self, opt):
        super().__init__(opt)
        self.net_g = build_network(opt['network_g'])
        self.net_g = self.model_to_device(self.net_g)
        self.print_network(self.net_g)
        load_path = self.opt.get('path', {}).get('pretrain_network_g', None)
        if load_path is not None:
            param_key = self.opt['path'].get('param_key_g', 'params')
            self.load_network(self.net_g, load_path, self.opt['path'].get('strict_load_g', True), param_key)
        if self.is_train:
            self.init_training_settings()

    def init_training_settings(self):
        self.net_g.train()
        train_opt = self.opt['train']
        self.use_amp = bool(train_opt.get('use_amp', False))
        if self.use_amp:
            # the reference's AMP is fp16 autocast + GradScaler (basicsr/models/srrs_model.py:28-31,
            # 79-82); the HIP kernels compute bf16 (no fp16 path, no loss scaling needed)
            get_root_logger().warning('train.use_amp: autocast runs in bfloat16 on the HIP kernels '
                                      '(the reference uses float16 + GradScaler; DESIGN.md §0)')
        self._graph = None
        self._eager_steps = 0
        # HIP-graph capture of the train step (after 2 eager warm-up steps); distributed: a chain of
        # graphs cut at the gradient buckets, all-reduced between them (utils/step_graph.py)
        self.use_graph = bool(train_opt.get('cuda_graph', False))
        # weight gradients on a side stream during backward (train.async_wgrad, ops.conv.async_wgrad);
        # the environment variable SR_ASYNC_WGRAD=0/1 overrides the option (A/B)
        env = switch('SR_ASYNC_WGRAD')
        mode = train_opt.get('async_wgrad', False)
        self.async_wgrad = {'0': False, '1': True, 'reduce': 'reduce'}.get(env, mode if mode == 'reduce' else bool(mode))
        if self.async_wgrad and self.opt.get('dist', False) and env != '1':
            from ..utils.dist_util import get_dist_info
            world = get_dist_info()[1]
            if world > max(1, torch.cuda.device_count()):
                # several ranks on one GPU (a gloo rehearsal): their side-stream graphs with
                # cross-queue waits stall each other for seconds per step
                get_root_logger().warning(f'train.async_wgrad disabled: {world} ranks share '
                                          f'{torch.cuda.device_count()} GPU(s)')
                self.async_wgrad = False
        # blocks whose side-stream launches share one fork (train.async_wgrad_blocks, ops.conv.side_batch;
        # SR_SIDE_BATCH overrides); applied only inside this model's backward (async_wgrad(blocks=))
        self.async_blocks = int(switch('SR_SIDE_BATCH') or train_opt.get('async_wgrad_blocks', 1))
        self.ema_decay = train_opt.get('ema_decay', 0)
        if self.ema_decay > 0:
            self.net_g_ema = build_network(self.opt['network_g']).to(self.device)
            self.flat_ema = FlatParams(self.net_g_ema, with_grad=False)
            load_path = self.opt.get('path', {}).get('pretrain_network_g', None)
            if load_path is not None:
                self.load_network(self.net_g_ema, load_path, self.opt['path'].get('strict_load_g', True), 'params_ema')
            else:
                self.model_ema(0)
            self.net_g_ema.eval()
        self.cri_pix = self.build_optional_loss(train_opt, 'pixel_opt')
        self.cri_perceptual = self.build_optional_loss(train_opt, 'perceptual_opt')
        if self.cri_pix is None and self.cri_perceptual is None:
            raise ValueError('Both pixel and perceptual losses are None.')
        self.setup_optimizers()
        self.setup_schedulers()

    def setup_optimizers(self):
        train_opt = self.opt['train']
        optim_opt = dict(train_opt['optim_g'])
        optim_type = optim_opt.pop('type')
        self.optimizer_g = self.get_optimizer(optim_type, self.flat_g.params, **optim_opt)
        self.optimizers.append(self.optimizer_g)

    def feed_data(self, data):
        # plain assignment also when a step is captured: the graph's static inputs live under
        # private names (_g_lq / _g_gt) and are refilled by optimize_parameters, so validation
        # batches of any shape never touch them
        self.lq = data['lq'].to(self.device, non_blocking=True)
        if 'gt' in data:
            self.gt = data['gt'].to(self.device, non_blocking=True)

    def _fused_step(self):
        return hasattr(self.optimizer_g, 'device_step')

    def _step_body(self, before_backward=None):
        """Device work of one train step (everything a captured replay re-executes).
        ``before_backward(loss) -> loss`` runs between the loss and backward (the segmented
        capture ends its forward segment there, utils/step_graph.py)."""
        self.optimizer_g.zero_grad()
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=self.use_amp):
            self.output = self.net_g(self.lq)
        l_total = 0
        loss_dict = OrderedDict()
        if self.cri_pix:
            l_pix = self.cri_pix(self.output, self.gt)
            l_total += l_pix
            loss_dict['l_pix'] = l_pix
        if before_backward is not None:
            l_total = before_backward(l_total)
        # weight gradients on a side stream, joined here
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
        # drop the autograd graph now: a graph kept alive by self.output would pin this step's
        # AccumulateGrad nodes (and their stream) into the next step / a HIP-graph capture
        self.output = self.output.detach()
        return loss_dict

    def _graph_inputs_match(self):
        return (self.lq.shape == self._g_lq.shape and self.lq.dtype == self._g_lq.dtype
                and self.gt.shape == self._g_gt.shape and self.gt.dtype == self._g_gt.dtype)

    def optimize_parameters(self, current_iter):
        if self._graph is not None and self._graph_inputs_match():
            if self.lq is not self._g_lq:
                self._g_lq.copy_(self.lq, non_blocking=True)
            if self.gt is not self._g_gt:
                self._g_gt.copy_(self.gt, non_blocking=True)
            self.optimizer_g.host_step()
            self._graph.replay()
            # the replay updated the parameters: host-side weight-image caches are now stale
            # (an eager forward, e.g. validation, rebuilds them in place)
            bump_param_epoch()
            self.output = self._g_out
            self.log_dict = self.reduce_loss_dict(self._graph_losses)
            return
        if self.use_graph and self._graph is None and self._eager_steps >= 2:
            self._capture_step()
            return
        loss_dict = self._step_body()
        self.sync_gradients()
        if self._fused_step():
            ema = self.flat_ema if self.ema_decay > 0 else None
            self.optimizer_g.step(ema=ema, ema_decay=self.ema_decay)
        else:
            self.optimizer_g.step()
            if self.ema_decay > 0:
                self.model_ema(decay=self.ema_decay)
        self._eager_steps += 1
        self.log_dict = self.reduce_loss_dict(loss_dict)

    def _capture_step(self):
        """Capture one whole train step (forward, L1, backward, fused Adam+EMA) in a HIP graph
        and run it; later steps replay it (train.cuda_graph).  Host-side per-step state (step
        count, lr) is kept outside the graph (FusedAdam.host_step + device hyper-parameters),
        the inputs live in static buffers refilled by feed_data.  Distributed: the step becomes
        a chain of graphs cut where the gradient buckets complete, with each bucket's all-reduce
        launched between them (utils/step_graph.py), so the exchange still overlaps backward."""
        torch.cuda.synchronize()
        ema = self.flat_ema if self.ema_decay > 0 else None
        self.optimizer_g.host_step()
        # the captured step reads these two tensors at replay: keep them under private names
        self._g_lq, self._g_gt = self.lq, self.gt

        def opt_step():
            self.optimizer_g.device_step(ema=ema, ema_decay=self.ema_decay)

        if isinstance(self.net_g, SRDistributed):
            g = SegmentedStepGraph(self.net_g.reducer, self.device)
            losses = g.capture(self._step_body, opt_step)
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                losses = self._step_body()
                opt_step()
        # the batched weight-image refresh inside the graph launches on these device tables
        self._graph_keep = take_captured_tables()
        self._graph = g
        self._g_out = self.output
        self._graph_losses = losses
        g.replay()
        self.log_dict = self.reduce_loss_dict(losses)

    def test(self):
        net = self.net_g_ema if hasattr(self, 'net_g_ema') else self.net_g
        was_training = self.net_g.training
        net.eval()
        with torch.no_grad():
            self.output = net(self.lq)
        if net is self.net_g and was_training:
            self.net_g.train()

    def nondist_validation(self, dataloader, current_iter, tb_logger, save_img):
        dataset_name = dataloader.dataset.opt['name']
        with_metrics = self.opt['val'].get('metrics') is not None
        if with_metrics:
            if not hasattr(self, 'metric_results'):
                self.metric_results = {metric: 0 for metric in self.opt['val']['metrics'].keys()}
            self._initialize_best_metric_results(dataset_name)
            self.metric_results = {metric: 0 for metric in self.metric_results}
        metric_data = dict()
        idx = -1
        for idx, val_data in enumerate(dataloader):
            img_name = osp.splitext(osp.basename(val_data['lq_path'][0]))[0] if 'lq_path' in val_data else str(idx)
            self.feed_data(val_data)
            self.test()
            visuals = self.get_current_visuals(current_iter)
            sr_img = tensor2img([visuals['result']])
            metric_data['img'] = sr_img
            if 'gt' in visuals:
                metric_data['img2'] = tensor2img([visuals['gt']])
                del self.gt
            del self.lq
            del self.output
            if save_img:
                imwrite(sr_img, self._val_image_path(dataset_name, img_name, current_iter))
            if with_metrics:
                for name, opt_ in self.opt['val']['metrics'].items():
                    self.metric_results[name] += calculate_metric(metric_data, opt_)
        if with_metrics:
            for metric in self.metric_results.keys():
                self.metric_results[metric] /= (idx + 1)
                self._update_best_metric_result(dataset_name, metric, self.metric_results[metric], current_iter)
            self._log_validation_metric_values(current_iter, dataset_name, tb_logger)

    def _val_image_path(self, dataset_name, img_name, current_iter):
        """Where a validation SR image goes (basicsr/models/sr_model.py:226-235): per image and
        iteration while training; per dataset with ``val.suffix`` (else the run name) at test time."""
        root = self.opt['path']['visualization']
        if self.opt['is_train']:
            return osp.join(root, img_name, f'{img_name}_{current_iter}.png')
        tag = self.opt['val'].get('suffix') or self.opt['name']
        return osp.join(root, dataset_name, f'{img_name}_{tag}.png')

    def _log_validation_metric_values(self, current_iter, dataset_name, tb_logger):
        """One log record with every metric and its best value / iteration, and a tensorboard
        scalar per metric (basicsr/models/sr_model.py:252-266)."""
        best = getattr(self, 'best_metric_results', {}).get(dataset_name, {})
        lines = [f'Validation {dataset_name}']
        for metric, value in self.metric_results.items():
            line = f'\t # {metric}: {value:.4f}'
            if metric in best:
                line += f'\tBest: {best[metric]["val"]:.4f} @ {best[metric]["iter"]} iter'
            lines.append(line)
        get_root_logger().info('\n'.join(lines) + '\n')
        if tb_logger:
            for metric, value in self.metric_results.items():
                tb_logger.add_scalar(f'metrics/{dataset_name}/{metric}', value, current_iter)

    def get_current_visuals(self, current_iter=None):
        out_dict = OrderedDict()
        out_dict['lq'] = self.lq.detach().cpu()
        out_dict['result'] = self.output.detach().float().cpu()
        if hasattr(self, 'gt'):
            out_dict['gt'] = self.gt.detach().cpu()
        return out_dict

    def save(self, epoch, current_iter):
        if hasattr(self, 'net_g_ema'):
            self.save_network([self.net_g, self.net_g_ema], 'net_g', current_iter, param_key=['params', 'params_ema'])
        else:
            self.save_network(self.net_g, 'net_g', current_iter)
        self.save_training_state(epoch, current_iter)
