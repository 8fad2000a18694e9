"""Drop-in `src/inference.py`: the reference's module path (`from src.inference import RestorationPipeline`,
app.py:18, scripts/generate_predictions.py:10) re-exported from the native MI355X engine package."""
import sys
from pathlib import Path

try:
    import image_restoration_and_enhancement_amd  # noqa: F401
except ImportError:  # repository layout: the package sits next to src/
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from image_restoration_and_enhancement_amd.inference import (  # noqa: E402,F401
    INPAINT_SIZE, NativeSDModel, RestorationPipeline, SD_PARAMS, TASK_MODEL_DIRS, Task, logger)

__all__ = ["RestorationPipeline", "TASK_MODEL_DIRS", "Task", "NativeSDModel"]
