"""Path pairing helpers (basicsr/data/data_util.py:200-291): folder scan and meta-info file."""
import os.path as osp

from ..utils.img_util import scandir


def paired_paths_from_folder(folders, keys, filename_tmpl):
    assert len(folders) == 2 and len(keys) == 2, 'folders / keys must be [input, gt]'
    input_folder, gt_folder = folders
    input_key, gt_key = keys
    input_paths = list(scandir(input_folder))
    gt_paths = list(scandir(gt_folder))
    assert len(input_paths) == len(gt_paths), (f'{input_key} and {gt_key} datasets have different number of images: '
                                               f'{len(input_paths)}, {len(gt_paths)}.')
    inputs = set(input_paths)
    paths = []
    for gt_path in gt_paths:
        base, ext = osp.splitext(osp.basename(gt_path))
        input_name = f'{filename_tmpl.format(base)}{ext}'
        assert input_name in inputs, f'{input_name} is not in {input_key}_paths.'
        paths.append({f'{input_key}_path': osp.join(input_folder, input_name),
                      f'{gt_key}_path': osp.join(gt_folder, gt_path)})
    return paths


def paired_paths_from_meta_info_file(folders, keys, meta_info_file, filename_tmpl):
    input_folder, gt_folder = folders
    input_key, gt_key = keys
    with open(meta_info_file, 'r') as fin:
        gt_names = [line.strip().split(' ')[0] for line in fin]
    paths = []
    for gt_name in gt_names:
        base, ext = osp.splitext(osp.basename(gt_name))
        input_name = f'{filename_tmpl.format(base)}{ext}'
        paths.append({f'{input_key}_path': osp.join(input_folder, input_name),
                      f'{gt_key}_path': osp.join(gt_folder, gt_name)})
    return paths


def paths_from_folder(folder):
    return [osp.join(folder, p) for p in scandir(folder)]
