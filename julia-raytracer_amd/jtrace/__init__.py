"""jtrace — host side of the MI355X path-tracing hot path (mirror of the reference's Jtrace
module surface: Cli, Scene/SceneIO, Bvh, Trace). The compute path is libjtrace_hip.so."""
from .abi import load_library, SceneABI, make_params  # noqa: F401
from .cli import Params, parse_cli_args  # noqa: F401
from .scene import find_camera  # noqa: F401
from .sceneio import load_scene, save_image  # noqa: F401
from .trace import (TraceState, make_scene_bvh, make_trace_lights, make_trace_state,  # noqa: F401
                    trace_samples, get_image)
