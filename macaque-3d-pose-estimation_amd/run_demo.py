"""run_demo.proc mirror (reference run_demo.py:21-39) for the 2D->3D hot path.

The reference chains step 1 (detect / track / pose / ID) -> step 2 (cross-view association) ->
step 3 (cross-frame association, kp2d.pickle) -> step 4 (2D filter + 3D lift) -> visualisation,
and imports the Cython ``pictorial`` module (run_demo.py:3-11) that no step calls.

This build runs the same chain on MI355X with the parts outside its scope replaced by data:

* step 1 (``src.pipeline.step1_proc2d.proc``): the pose slice over every camera's frame store;
  the detector / tracker / ID classifier output arrives as the stores' tracker rows;
* steps 2-3: association is bypassed -- ``kp2d.pickle`` is written by step 3's own
  ``create_kp2dfile`` from a known track -> individual map
  (``src.pipeline.step3_crossframematching.proc_known_assignment``);
* step 4 (``src.pipeline.step4_aniposefiltering.proc``): unchanged drop-in;
* visualisation (video rendering) is out of scope and the ``pictorial`` import is not needed.
"""
from src.pipeline import step1_proc2d as step1
from src.pipeline import step3_crossframematching as step3
from src.pipeline import step4_aniposefiltering as step4


def proc(data_name, fps, results_dir_root, device_str, config_path, raw_data_dir, n_kp, vidfile_prefix='',
         n_animal=4, track_to_animal=None, pose_model=None):
    """run_demo.py:21-30: step 1 -> (known assignment) -> step 4; returns step 4's kp3d dict."""
    device = int(device_str.split(':')[1]) if ':' in device_str else 0
    step1.proc(data_name, results_dir_root, raw_data_dir, device_str, fps, pose_model=pose_model)
    step3.proc_known_assignment(data_name, results_dir_root, config_path, n_animal=n_animal, n_kp=n_kp,
                                track_to_animal=track_to_animal)
    return step4.proc(data_name, results_dir_root, config_path, n_kp, redo=True, device=device)


if __name__ == '__main__':
    proc('example', 24, './results3D', 'cuda:0', './calib/config.yaml', './videos', 17)
