"""PairedImageDataset (basicsr/data/paired_image_dataset.py:10-106): LQ/GT pairs from folders
or a meta-info file, random paired crop + flip/rotation in the train phase, BGR -> RGB CHW
float32 in [0, 1], optional mean/std normalisation.  ``io_backend`` 'disk' (the lmdb backend
needs the lmdb package, which this image lacks: it raises with that message)."""
import torch
from torch.utils import data as data

from ..utils.img_util import img2tensor, imfrombytes
from ..utils.registry import DATASET_REGISTRY
from .data_util import paired_paths_from_folder, paired_paths_from_meta_info_file
from .transforms import augment, paired_random_crop


class FileClient:
    """Disk file client (basicsr/utils/file_client.py: the 'disk' backend)."""

    def __init__(self, backend='disk', **kwargs):
        if backend != 'disk':
            raise NotImplementedError(f'io backend {backend!r} is not available in this build (only "disk")')

    def get(self, filepath, client_key=None):
        with open(filepath, 'rb') as f:
            return f.read()


def _bgr2y(img):
    """Y channel of BT.601 (bgr2ycbcr y_only, basicsr/utils/color_util.py:60-84) for [0, 1] floats."""
    return (img @ [24.966, 128.553, 65.481] + 16.0) / 255.


@DATASET_REGISTRY.register()
class PairedImageDataset(data.Dataset):

    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        self.file_client = None
        self.io_backend_opt = dict(opt['io_backend'])
        self.mean = opt.get('mean')
        self.std = opt.get('std')
        self.gt_folder, self.lq_folder = opt['dataroot_gt'], opt['dataroot_lq']
        self.filename_tmpl = opt.get('filename_tmpl', '{}')
        if self.io_backend_opt['type'] == 'lmdb':
            raise NotImplementedError('lmdb io backend: the lmdb package is not available in this build')
        if opt.get('meta_info_file') is not None:
            self.paths = paired_paths_from_meta_info_file([self.lq_folder, self.gt_folder], ['lq', 'gt'],
                                                          opt['meta_info_file'], self.filename_tmpl)
        else:
            self.paths = paired_paths_from_folder([self.lq_folder, self.gt_folder], ['lq', 'gt'], self.filename_tmpl)

    def __getitem__(self, index):
        if self.file_client is None:
            opt = dict(self.io_backend_opt)
            self.file_client = FileClient(opt.pop('type'), **opt)
        scale = self.opt['scale']
        gt_path = self.paths[index]['gt_path']
        lq_path = self.paths[index]['lq_path']
        img_gt = imfrombytes(self.file_client.get(gt_path, 'gt'), float32=True)
        img_lq = imfrombytes(self.file_client.get(lq_path, 'lq'), float32=True)
        if self.opt['phase'] == 'train':
            img_gt, img_lq = paired_random_crop(img_gt, img_lq, self.opt['gt_size'], scale, gt_path)
            img_gt, img_lq = augment([img_gt, img_lq], self.opt['use_hflip'], self.opt['use_rot'])
        if self.opt.get('color') == 'y':
            img_gt = _bgr2y(img_gt)[..., None].astype('float32')
            img_lq = _bgr2y(img_lq)[..., None].astype('float32')
        if self.opt['phase'] != 'train':
            img_gt = img_gt[0:img_lq.shape[0] * scale, 0:img_lq.shape[1] * scale, :]
        img_gt, img_lq = img2tensor([img_gt, img_lq], bgr2rgb=True, float32=True)
        if self.mean is not None or self.std is not None:
            for t in (img_lq, img_gt):
                m = torch.tensor(self.mean if self.mean is not None else [0.] * t.shape[0]).view(-1, 1, 1)
                s = torch.tensor(self.std if self.std is not None else [1.] * t.shape[0]).view(-1, 1, 1)
                t.sub_(m).div_(s)
        return {'lq': img_lq, 'gt': img_gt, 'lq_path': lq_path, 'gt_path': gt_path}

    def __len__(self):
        return len(self.paths)
