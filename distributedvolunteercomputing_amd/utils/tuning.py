"""Library-GEMM selection for the MI355X (gfx950) bench shapes.

The plain GEMMs of the transformer (projections, MLP, LM head) are library GEMMs
(hipBLASLt / rocBLAS). PyTorch's TunableOp benchmarks every candidate solution of both
libraries for each GEMM shape; `scripts/gpu_tune.sh` runs it on an MI355X and the winners
are committed in ``tuning/tunableop_gfx950.csv``. At run time we only LOOK UP those results
(tuning disabled), so a fresh box gets the tuned kernels with no tuning cost.

Must be called before torch issues its first GEMM (it only sets environment variables).
Set VCX_TUNABLEOP=off to disable; VCX_TUNABLEOP_FILE=<csv> to use another results file.
"""
from __future__ import annotations

import os
import shutil
import tempfile

from .. import config

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
RESULTS = os.path.join(ROOT, "tuning", "tunableop_gfx950.csv")


def enable_tuned_gemms(local_rank: int = 0) -> bool:
    cfg = config.get()
    if cfg.tunableop == "off" or "PYTORCH_TUNABLEOP_ENABLED" in os.environ:
        return False
    results = cfg.tunableop_file or RESULTS
    if not os.path.exists(results):
        return False
    d = tempfile.mkdtemp(prefix="vcx_tunableop_")
    # TunableOp keys its results file by device ordinal; give this rank its own copy
    shutil.copyfile(results, os.path.join(d, f"results{local_rank}.csv"))
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "0"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.join(d, "results%d.csv")
    return True
