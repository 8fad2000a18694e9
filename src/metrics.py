"""Drop-in `src/metrics.py` (scripts/evaluate_model.py:14) re-exported from the numpy/scipy restatement
`image_restoration_and_enhancement_amd.metrics` (no cv2 / scikit-image / torchvision needed)."""
import sys
from pathlib import Path

try:
    import image_restoration_and_enhancement_amd  # noqa: F401
except ImportError:
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from image_restoration_and_enhancement_amd.metrics import (  # noqa: E402,F401
    FID_AVAILABLE, LPIPS_AVAILABLE, MetricsCalculator, evaluate_task, load_image, print_results)
