"""Action-conditioned plumbing on the CPU: relative-action extraction and rotation helpers
(restated from the reference's action_conditioned.py:62-135 and dataset_utils.py; no golden vectors
ship with the reference for these, so the checks are the defining properties: parity unpinned)."""
import numpy as np
import pytest

from cosmos_predict2.action_conditioned import (euler2rotm, get_action_sequence_from_states, relative_actions,
                                                rotm2euler, rotm2quat)
from cosmos_predict2.net_config import MODELS


def test_euler_roundtrip_and_quat():
    rng = np.random.RandomState(0)
    for _ in range(50):
        e = rng.uniform(-np.pi, np.pi, 3)
        e[1] = rng.uniform(-1.4, 1.4)  # away from the pitch singularity
        R = euler2rotm(e)
        assert np.allclose(R.T @ R, np.eye(3), atol=1e-12)
        assert np.allclose(euler2rotm(rotm2euler(R)), R, atol=1e-9)
        q = rotm2quat(R)
        assert abs(np.linalg.norm(q) - 1) < 1e-9


def test_relative_actions_frame_and_gripper():
    # a robot yawed by 90 degrees moving along world +y moves along its own +x
    arm = np.array([[0, 0, 0, 0, 0, np.pi / 2], [0, 1, 0, 0, 0, np.pi / 2], [0, 1, 0, 0, 0, np.pi / 2]], float)
    grip = np.array([0.0, 0.5, 1.0])
    a = relative_actions(arm, grip)
    assert a.shape == (2, 7)
    assert np.allclose(a[0, :3], [1, 0, 0], atol=1e-12)
    assert np.allclose(a[0, 3:6], 0, atol=1e-12) and np.allclose(a[1, :6], 0, atol=1e-12)
    assert a[0, 6] == 0.5 and a[1, 6] == 1.0
    s = get_action_sequence_from_states({"state": arm, "continuous_gripper_state": grip}, action_scaler=20.0,
                                        gripper_scale=2.0)
    assert np.allclose(s[0, :3], [20, 0, 0]) and s[1, 6] == 2.0


def test_action_model_registered():
    net, samp = MODELS["2B/robot/action-cond"]
    assert net.action_dim == 7 and net.action_per_latent_frame == 4 and net.action_in_features == 28
    assert samp.state_t == 4  # 13 frames per chunk of 12 actions
    with pytest.raises(NotImplementedError):
        get_action_sequence_from_states({"state": np.zeros((3, 6)), "continuous_gripper_state": np.zeros(3)},
                                        use_quat=True)


def test_multiview_model_registered():
    net, samp = MODELS["2B/auto/multiview"]
    assert net.n_cameras_emb == 7 and net.view_condition_dim == 7 and net.state_t == 8
    assert net.patch_features == (16 + 1 + 1 + 7) * 4  # x_embedder [2048, 100]
    assert samp.cfg_mode == "text2world"
    from cosmos_predict2.dit import state_dict_shapes

    s = state_dict_shapes(net)
    assert s["x_embedder.proj.1.weight"][0] == (2048, 100) and s["view_embeddings.weight"][0] == (7, 7)
