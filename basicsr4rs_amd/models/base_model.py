"""Model base class (mirror of basicsr/models/base_model.py:13-401).

Same method contract as the reference (the train loop of basicsr/train.py:126-209 and
tests/test_models/test_sr_model.py drive these): optimizers/schedulers from the options
dict, ``update_learning_rate`` with warm-up, ``model_ema``, ``save_network`` /
``load_network`` ({param_key: state_dict}, 'module.' stripped, strict by default),
``save_training_state`` / ``resume_training``, ``reduce_loss_dict``.

MI355X-specific parts: ``model_to_device`` moves the net, re-points its parameters into a
flat fp32 buffer (utils/flat.py) and, when distributed, attaches the bucketed RCCL
gradient reducer instead of torch's DistributedDataParallel; ``reduce_loss_dict`` is
deferred until the log is read (no host sync inside optimize_parameters).
"""
import os
import time
from collections import OrderedDict
from copy import deepcopy

import torch
import torch.distributed as dist
from torch import nn

from ..utils.dist_util import get_dist_info, master_only
from ..utils.flat import FlatParams, FusedAdam, GradBucketReducer
from . import lr_scheduler as lr_scheduler


class SRDistributed(nn.Module):
    """DDP-equivalent wrapper: ``.module`` is the bare net; gradients are averaged by the
    reducer (launched from backward hooks, joined in ``BaseModel.sync_gradients``)."""

    def __init__(self, module, flat, bucket_mb=25.0, find_unused_parameters=False):
        super().__init__()
        self.module = module
        self.reducer = GradBucketReducer(flat, bucket_mb=bucket_mb, find_unused=find_unused_parameters)
        self.reducer.broadcast_params(0)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)


class BaseModel:

    def __init__(self, opt):
        self.opt = opt
        self.device = torch.device('cuda' if opt.get('num_gpu', 1) != 0 else 'cpu')
        self.is_train = opt['is_train']
        self.schedulers = []
        self.optimizers = []
        self.flat_g = None
        self.flat_ema = None
        self._graph = None
        self._pending_losses = None
        self.log_dict = OrderedDict()

    def feed_data(self, data):
        pass

    def optimize_parameters(self, current_iter):
        pass

    def get_current_visuals(self, current_iter=None):
        pass

    def save(self, epoch, current_iter):
        pass

    def validation(self, dataloader, current_iter, tb_logger, save_img=False):
        if self.opt.get('dist', False):
            self.dist_validation(dataloader, current_iter, tb_logger, save_img)
        else:
            self.nondist_validation(dataloader, current_iter, tb_logger, save_img)

    def dist_validation(self, dataloader, current_iter, tb_logger, save_img):
        if get_dist_info()[0] == 0:
            self.nondist_validation(dataloader, current_iter, tb_logger, save_img)

    def _initialize_best_metric_results(self, dataset_name):
        if hasattr(self, 'best_metric_results') and dataset_name in self.best_metric_results:
            return
        if not hasattr(self, 'best_metric_results'):
            self.best_metric_results = dict()
        record = dict()
        for metric, content in self.opt['val']['metrics'].items():
            better = content.get('better', 'higher')
            record[metric] = dict(better=better, val=float('-inf') if better == 'higher' else float('inf'), iter=-1)
        self.best_metric_results[dataset_name] = record

    def _update_best_metric_result(self, dataset_name, metric, val, current_iter):
        rec = self.best_metric_results[dataset_name][metric]
        if (rec['better'] == 'higher' and val >= rec['val']) or (rec['better'] != 'higher' and val <= rec['val']):
            rec['val'] = val
            rec['iter'] = current_iter

    def model_ema(self, decay=0.999):
        """p_ema = decay * p_ema + (1 - decay) * p over named parameters (base_model.py:75-82)."""
        net_g = self.get_bare_model(self.net_g)
        net_g_params = dict(net_g.named_parameters())
        with torch.no_grad():
            for k, v in self.net_g_ema.named_parameters():
                v.data.mul_(decay).add_(net_g_params[k].data, alpha=1 - decay)
        from ..ops.conv import bump_param_epoch
        bump_param_epoch()

    def get_current_log(self):
        if self._pending_losses is not None:
            self.log_dict = self._finish_reduce(self._pending_losses)
            self._pending_losses = None
        return self.log_dict

    def model_to_device(self, net):
        """Move to the device, flatten the parameters, attach the gradient reducer (DDP)."""
        net = net.to(self.device)
        if self.is_train:
            self.flat_g = FlatParams(net)
        if self.opt.get('dist', False):
            bucket_mb = self.opt.get('bucket_cap_mb', 25.0)
            # base_model.py:96-99 passes find_unused_parameters to DDP
            net = SRDistributed(net, self.flat_g, bucket_mb=bucket_mb,
                                find_unused_parameters=self.opt.get('find_unused_parameters', False))
        return net

    def sync_gradients(self):
        """Join the bucketed all-reduces; the 1/world average is applied by the optimizer."""
        if isinstance(self.net_g, SRDistributed):
            self.net_g.reducer.wait()
            world = dist.get_world_size()
            for o in self.optimizers:
                if isinstance(o, FusedAdam):
                    o.grad_scale = 1.0 / world

    def get_optimizer(self, optim_type, params, lr, **kwargs):
        if optim_type == 'Adam' and self.flat_g is not None and params is self.flat_g.params:
            return FusedAdam(self.flat_g, lr, **kwargs)
        optimizers = {
            'Adam': torch.optim.Adam,
            'AdamW': torch.optim.AdamW,
            'Adamax': torch.optim.Adamax,
            'SGD': torch.optim.SGD,
            'ASGD': torch.optim.ASGD,
            'RMSprop': torch.optim.RMSprop,
            'Rprop': torch.optim.Rprop
        }
        if optim_type not in optimizers:
            raise NotImplementedError(f'optimizer {optim_type} is not supported yet.')
        return optimizers[optim_type](params, lr, **kwargs)

    def setup_schedulers(self):
        train_opt = self.opt['train']
        scheduler_type = train_opt['scheduler'].pop('type')
        if scheduler_type in ['MultiStepLR', 'MultiStepRestartLR']:
            cls = lr_scheduler.MultiStepRestartLR
        elif scheduler_type == 'CosineAnnealingRestartLR':
            cls = lr_scheduler.CosineAnnealingRestartLR
        else:
            raise NotImplementedError(f'Scheduler {scheduler_type} is not implemented yet.')
        for optimizer in self.optimizers:
            self.schedulers.append(cls(optimizer, **train_opt['scheduler']))

    def get_bare_model(self, net):
        if isinstance(net, (SRDistributed, nn.parallel.DistributedDataParallel, nn.DataParallel)):
            net = net.module
        return net

    @master_only
    def print_network(self, net):
        net = self.get_bare_model(net)
        n = sum(p.numel() for p in net.parameters())
        print(f'Network: {net.__class__.__name__}, with parameters: {n:,d}')

    def _set_lr(self, lr_groups_l):
        for optimizer, lr_groups in zip(self.optimizers, lr_groups_l):
            for param_group, lr in zip(optimizer.param_groups, lr_groups):
                param_group['lr'] = lr

    def _get_init_lr(self):
        return [[v['initial_lr'] for v in optimizer.param_groups] for optimizer in self.optimizers]

    def update_learning_rate(self, current_iter, warmup_iter=-1):
        """Scheduler step each iteration; linear warm-up below ``warmup_iter`` (base_model.py:185-206)."""
        if current_iter > 1:
            for scheduler in self.schedulers:
                scheduler.step()
        if current_iter < warmup_iter:
            init_lr_g_l = self._get_init_lr()
            self._set_lr([[v / warmup_iter * current_iter for v in g] for g in init_lr_g_l])

    def get_current_learning_rate(self):
        return [param_group['lr'] for param_group in self.optimizers[0].param_groups]

    @master_only
    def save_network(self, net, net_label, current_iter, param_key='params'):
        current_iter = 'latest' if current_iter == -1 else current_iter
        save_path = os.path.join(self.opt['path']['models'], f'{net_label}_{current_iter}.pth')
        net = net if isinstance(net, list) else [net]
        param_key = param_key if isinstance(param_key, list) else [param_key]
        assert len(net) == len(param_key), 'The lengths of net and param_key should be the same.'
        save_dict = {}
        for net_, key_ in zip(net, param_key):
            net_ = self.get_bare_model(net_)
            state_dict = net_.state_dict()
            save_dict[key_] = OrderedDict(
                (k[7:] if k.startswith('module.') else k, v.detach().cpu()) for k, v in state_dict.items())
        for retry in range(3):  # avoid occasional writing errors (base_model.py:241-256)
            try:
                torch.save(save_dict, save_path)
                break
            except Exception as e:  # pragma: no cover
                print(f'Save model error: {e}, remaining retry times: {2 - retry}')
                time.sleep(1)

    def load_network(self, net, load_path, strict=True, param_key='params'):
        net = self.get_bare_model(net)
        load_net = torch.load(load_path, map_location='cpu', weights_only=True)
        if param_key is not None:
            if param_key not in load_net and 'params' in load_net:
                param_key = 'params'
            load_net = load_net[param_key]
        load_net = OrderedDict((k[7:] if k.startswith('module.') else k, v) for k, v in load_net.items())
        if not strict:
            crt = net.state_dict()
            for k in list(load_net.keys()):
                if k in crt and crt[k].size() != load_net[k].size():
                    load_net[k + '.ignore'] = load_net.pop(k)
        with torch.no_grad():
            net.load_state_dict(load_net, strict=strict)
        from ..ops.conv import bump_param_epoch
        bump_param_epoch()

    def get_training_state(self, epoch, current_iter):
        return {
            'epoch': epoch,
            'iter': current_iter,
            'optimizers': [o.state_dict() for o in self.optimizers],
            'schedulers': [s.state_dict() for s in self.schedulers]
        }

    @master_only
    def save_training_state(self, epoch, current_iter):
        if current_iter != -1:
            state = self.get_training_state(epoch, current_iter)
            save_path = os.path.join(self.opt['path']['training_states'], f'{current_iter}.state')
            for retry in range(3):
                try:
                    torch.save(state, save_path)
                    break
                except Exception as e:  # pragma: no cover
                    print(f'Save training state error: {e}, remaining retry times: {2 - retry}')
                    time.sleep(1)

    def resume_training(self, resume_state):
        assert len(resume_state['optimizers']) == len(self.optimizers), 'Wrong lengths of optimizers'
        assert len(resume_state['schedulers']) == len(self.schedulers), 'Wrong lengths of schedulers'
        for o, s in zip(self.optimizers, resume_state['optimizers']):
            o.load_state_dict(s)
        for sch, s in zip(self.schedulers, resume_state['schedulers']):
            sch.load_state_dict(s)

    def reduce_loss_dict(self, loss_dict):
        """Average losses over ranks (base_model.py:376-401).  The reduction and the host
        read happen when the log is requested (get_current_log), not every iteration."""
        self._pending_losses = OrderedDict((k, v.detach()) for k, v in loss_dict.items())
        return self._pending_losses

    def _finish_reduce(self, loss_dict):
        with torch.no_grad():
            if self.opt.get('dist', False) and len(loss_dict):
                keys = list(loss_dict.keys())
                losses = torch.stack([loss_dict[k].float() for k in keys], 0)
                torch.distributed.reduce(losses, dst=0)
                if self.opt.get('rank', get_dist_info()[0]) == 0:
                    losses /= self.opt.get('world_size', get_dist_info()[1])
                loss_dict = dict(zip(keys, losses))
            return OrderedDict((k, v.mean().item()) for k, v in loss_dict.items())


def deep_opt(opt):
    return deepcopy(opt)
