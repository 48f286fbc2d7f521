"""run_demo.proc mirror (reference run_demo.py:21-39) for the hot path.

The reference chains step1 (detect/track/pose/ID) -> step2/3 (cross-view and
cross-frame association, incl. the Cython ``pictorial`` module it imports at
run_demo.py:6) -> step4 (2D filter + 3D lift) -> visualisation.  This build
implements the pose slice of step 1 and all of step 4 on MI355X; association,
detection, tracking and the visualiser are outside its scope, so
the pictorial import is simply not needed.  ``proc`` runs step 4 on a results
directory whose ``kp2d.pickle`` was produced upstream (by the reference's own
steps 1-3, or by this build's step-1 slice plus an external association).
"""
import os

from src.pipeline import step4_aniposefiltering as step4


def proc(data_name, fps, results_dir_root, device_str, config_path, raw_data_dir, n_kp, vidfile_prefix=''):
    kp2d = os.path.join(results_dir_root, data_name, 'kp2d.pickle')
    if not os.path.exists(kp2d):
        raise FileNotFoundError(f'{kp2d} not found: steps 1-3 (detection, tracking, association) run upstream '
                                'of this build')
    device = int(device_str.split(':')[1]) if ':' in device_str else 0
    return step4.proc(data_name, results_dir_root, config_path, n_kp, redo=True, device=device)


if __name__ == '__main__':
    proc('example', 24, './results3D', 'cuda:0', './calib/config.yaml', './videos', 17)
