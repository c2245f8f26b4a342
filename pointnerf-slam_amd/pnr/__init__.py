"""pnr -- MI355X-native drop-in for the render_batch_ray hot path of thua919/pointNeRF-SLAM.

Host mirror of the reference operator API (src/utils/Renderer.py, src/conv_onet/models/decoder.py,
src/config.py) over the C ABI of libpnr.so (include/pnr.h).  See DESIGN.md.
"""
from . import _lib
from .config import load_config, get_model, ROOM0_CFG
from .decoder import MLP, PARAM_ORDER, FC_ORDER
from .points import NeuralPoints
from .renderer import Renderer, get_rays, get_rays_from_uv, get_samples
from .common import scaled_bound, get_camera_from_tensor, get_tensor_from_camera, quad2rotation, random_select
from .tracking import TrackStep, track_frame
from . import mesher, logger
from .logger import Logger, load_ckpt

__all__ = ['Renderer', 'MLP', 'PARAM_ORDER', 'FC_ORDER', 'NeuralPoints', 'get_model', 'load_config', 'ROOM0_CFG', 'get_rays',
           'get_rays_from_uv', 'scaled_bound', 'get_camera_from_tensor', 'get_tensor_from_camera',
           'quad2rotation', 'TrackStep', 'track_frame', 'get_samples', 'random_select', 'mesher', 'logger', 'Logger',
           'load_ckpt']


def library():
    """Load libpnr.so (raises if it was not built)."""
    return _lib.load()
