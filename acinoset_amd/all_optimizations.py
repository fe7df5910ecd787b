"""Drop-in for the reference's pipeline script `src/all_optimizations.py`:
the same command line, the same frame selection, the same `core.fte` call, on the GPU.

    python -m acinoset_amd.all_optimizations --data_dir DIR [--dlc dlc] [--start_frame 1]
        [--end_frame -1] [--dlc_thresh 0.8] [--plot] [--fps F] [--mode head]

What differs, and why:
* Video information (`app.get_vid_info`, `src/all_optimizations.py:48`) is read from the
  videos with OpenCV in the reference; OpenCV is absent here. The resolution is taken from the
  scene file (the reference asserts they agree, :67), the frame count from the DLC data (or
  `--num_frames`), and the frame rate from `--fps` (default 90, the AcinoSet cameras'
  rate).
* DLC files: `*.h5` as in the reference (pandas + PyTables), else DLC's `*.csv` export.
* `--mode` (default 'head', the reference's hard-coded value at :42).
"""
import os
from argparse import ArgumentParser
from glob import glob
from typing import List, Optional, Tuple

import numpy as np

from . import core
from .lib import misc, utils


def get_vid_info(data_dir: str, cam_res, points_2d_df, fps: float = 90.0, num_frames: Optional[int] = None):
    """(res, fps, num_frames, codec) like `app.get_vid_info` (`src/lib/app.py:350-367`)
    without the videos (see the module docstring)."""
    if num_frames is None:
        num_frames = int(points_2d_df['frame'].max()) + 1
    return tuple(cam_res), float(fps), int(num_frames), None


def auto_frame_range(filtered_points_2d_df, target_markers: List[str]) -> Tuple[int, int]:
    """`src/all_optimizations.py:79-113`: the first and the last frame in which every target
    marker is detected (likelihood above the threshold) by at least one camera. The reference
    scans frames 0 .. max and max .. 1 with one DataFrame query per frame; this counts the
    detected target markers of every frame once."""
    df = filtered_points_2d_df[filtered_points_2d_df['marker'].isin(target_markers)]
    max_idx = int(filtered_points_2d_df['frame'].max() + 1)
    n_markers = df.groupby('frame')['marker'].nunique()
    ok = set(int(f) for f in n_markers.index[n_markers.to_numpy() >= len(target_markers)])
    start_frame = next((i for i in range(max_idx) if i in ok), None)
    end_frame = next((i for i in range(max_idx, 0, -1) if i in ok), None)
    if start_frame is None or end_frame is None:
        raise RuntimeError('Setting frames failed. Please define start and end frames manually.')
    return start_frame, end_frame


def dlc_files(dlc_dir: str) -> List[str]:
    files = sorted(glob(os.path.join(dlc_dir, '*.h5')))
    return files if files else sorted(glob(os.path.join(dlc_dir, '*.csv')))


def main(argv=None) -> str:
    parser = ArgumentParser(description='AcinoSet optimisations on the MI355X (drop-in for all_optimizations.py)')
    parser.add_argument('--data_dir', type=str, help='The file path to the flick/run to be optimized.')
    parser.add_argument('--dlc', type=str, default='dlc', help='The DLC directory inside data_dir.')
    parser.add_argument('--start_frame', type=int, default=1,
                        help='The frame at which the optimized reconstruction will start.')
    parser.add_argument('--end_frame', type=int, default=-1,
                        help='The frame at which the optimized reconstruction will end. If it is -1, start_frame '
                             'and end_frame are automatically set.')
    parser.add_argument('--dlc_thresh', type=float, default=0.8,
                        help='The likelihood of the dlc points below which will be excluded from the optimization.')
    parser.add_argument('--plot', action='store_true', help='Show the plots (accepted; no plotting here).')
    parser.add_argument('--fps', type=float, default=90.0, help='Video frame rate (the videos are not read).')
    parser.add_argument('--num_frames', type=int, default=None, help='Video frame count (default: from DLC).')
    parser.add_argument('--mode', type=str, default='head', help="Marker mode ('head' in the reference).")
    args = parser.parse_args(argv)
    mode = args.mode

    DATA_DIR = os.path.normpath(args.data_dir)
    assert os.path.exists(DATA_DIR), f'Data directory not found: {DATA_DIR}'
    DLC_DIR = os.path.join(DATA_DIR, args.dlc)
    assert os.path.exists(DLC_DIR), f'DLC directory not found: {DLC_DIR}'

    # load scene data
    k_arr, d_arr, r_arr, t_arr, cam_res, n_cams, scene_fpath = utils.find_scene_file(DATA_DIR, verbose=False)
    camera_params = (k_arr, d_arr, r_arr, t_arr, cam_res, n_cams)
    # load DLC data
    dlc_points_fpaths = dlc_files(DLC_DIR)
    assert n_cams == len(dlc_points_fpaths), f'# of dlc files != # of cams in {n_cams}_cam_scene_sba.json'
    points_2d_df = utils.load_dlc_points_as_df(dlc_points_fpaths, frame_shifts=[0] * n_cams, verbose=False)
    filtered_points_2d_df = points_2d_df.query(f'likelihood > {args.dlc_thresh}')

    res, fps, num_frames, _ = get_vid_info(DATA_DIR, cam_res, points_2d_df, args.fps, args.num_frames)
    vid_params = {'vid_resolution': res, 'vid_fps': fps, 'total_frames': num_frames}
    assert 0 < args.start_frame < num_frames, f'start_frame must be strictly between 0 and {num_frames}'
    assert 0 != args.end_frame <= num_frames, f'end_frame must be less than or equal to {num_frames}'
    assert 0 <= args.dlc_thresh <= 1, 'dlc_thresh must be from 0 to 1'

    if args.end_frame == -1:
        start_frame, end_frame = auto_frame_range(filtered_points_2d_df, misc.get_markers(mode))
    else:
        start_frame = args.start_frame - 1  # 0 based indexing
        end_frame = args.end_frame
    assert len(k_arr) == points_2d_df['camera'].nunique()

    print('========== FTE ==========\n')
    OUT_DIR = os.path.join(DATA_DIR, 'fte')
    return core.fte(OUT_DIR, points_2d_df, mode, camera_params, start_frame, end_frame, args.dlc_thresh,
                    scene_fpath, params=vid_params, shutter_delay=True, shutter_delay_mode='const',
                    interpolation_mode='vel', video=True, plot=args.plot)


if __name__ == '__main__':
    main()
