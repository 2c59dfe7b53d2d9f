"""GPU: the trainer and the device replay ring against the reference's own outputs (G7 / G8).

* DeviceReplay.deduplicate on the device vs the reference's Deduplicator (memory_ops.json);
* _Trainer.train_batch on the device vs the reference's update_from_memory steps
  (trainer_step.npz) in the modes a GPU run can reproduce: "train_nodrop" (train-mode
  BatchNorm statistics, dropout p = 0) and "eval" — the "train" mode's dropout masks come from
  the CPU generator and are checked on the CPU (test_trainer_golden.py).  Tolerances are the CPU
  test's scaled by 20 (fp32 convolutions on the GPU sum in another order).
"""
import numpy as np
import pytest

from tests.parity_helpers import golden_path, load_json
from tests.test_memory_golden import check_device_dedup
from tests.test_trainer_golden import NETS, check_trainer

pytestmark = pytest.mark.gpu


def test_device_replay_deduplicate_on_gpu_matches_reference():
    check_device_dedup(load_json("memory_ops.json"), "cuda")


@pytest.mark.parametrize("name", list(NETS))
@pytest.mark.parametrize("mode", ["train_nodrop", "eval"])
def test_trainer_step_on_gpu_matches_reference(name, mode):
    check_trainer(dict(np.load(golden_path("trainer_step.npz"))), name, mode, "cuda", loose=20.0)
