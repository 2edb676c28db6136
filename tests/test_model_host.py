"""Host-side model logic that needs no device: validation image paths and the validation metric
record (basicsr/models/sr_model.py:226-235, :252-266)."""
import logging
from types import SimpleNamespace

from basicsr4rs_amd.models.sr_model import SRModel


def test_val_image_path_train_and_test():
    m = SimpleNamespace(opt=dict(is_train=True, name='run1', path=dict(visualization='/v'), val=dict()))
    assert SRModel._val_image_path(m, 'Set5', 'baby', 1000) == '/v/baby/baby_1000.png'
    m.opt['is_train'] = False
    assert SRModel._val_image_path(m, 'Set5', 'baby', 'x') == '/v/Set5/baby_run1.png'
    m.opt['val']['suffix'] = 'sfx'
    assert SRModel._val_image_path(m, 'Set5', 'baby', 'x') == '/v/Set5/baby_sfx.png'


def test_validation_metric_record():
    class TB:
        def __init__(self):
            self.rows = []

        def add_scalar(self, *a):
            self.rows.append(a)

    m = SimpleNamespace(metric_results={'psnr': 31.25, 'ssim': 0.9},
                        best_metric_results={'Set5': {'psnr': dict(val=32.0, iter=7), 'ssim': dict(val=0.91, iter=3)}})
    from basicsr4rs_amd.utils.logger import get_root_logger
    tb = TB()
    records = []
    h = logging.Handler()
    h.emit = lambda r: records.append(r.getMessage())
    lg = get_root_logger()
    lg.addHandler(h)
    try:
        SRModel._log_validation_metric_values(m, 10, 'Set5', tb)
    finally:
        lg.removeHandler(h)
    text = '\n'.join(records)
    assert 'Validation Set5' in text and '# psnr: 31.2500\tBest: 32.0000 @ 7 iter' in text
    assert '# ssim: 0.9000\tBest: 0.9100 @ 3 iter' in text
    assert tb.rows == [('metrics/Set5/psnr', 31.25, 10), ('metrics/Set5/ssim', 0.9, 10)]
