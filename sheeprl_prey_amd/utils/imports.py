"""Optional-dependency guards (reference: ``sheeprl/utils/imports.py:1-14``)."""
import importlib.util
import platform


def _available(name: str) -> bool:
    try:
        return importlib.util.find_spec(name) is not None
    except (ImportError, ValueError):
        return False


_IS_WINDOWS = platform.system() == "Windows"
_IS_ATARI_AVAILABLE = _available("ale_py")
_IS_ATARI_ROMS_AVAILABLE = _IS_ATARI_AVAILABLE
_IS_CRAFTER_AVAILABLE = _available("crafter")
_IS_DIAMBRA_AVAILABLE = _available("diambra")
_IS_DIAMBRA_ARENA_AVAILABLE = _available("diambra.arena") if _IS_DIAMBRA_AVAILABLE else False
_IS_DMC_AVAILABLE = _available("dm_control")
_IS_MINEDOJO_AVAILABLE = _available("minedojo")
_IS_MINERL_0_4_4_AVAILABLE = _available("minerl")
_IS_BOX2D_AVAILABLE = _available("Box2D")
_IS_CV2_AVAILABLE = _available("cv2")
_IS_TORCH_GREATER_EQUAL_2_0 = True
