"""pfml — MI355X-native Portfolio-ML (JKMP 2022) backtesting engine.

Stages (SURVEY §1 layer map), each importable and runnable from the CLI (``python -m pfml``):

=====================  ===============================  ==========================================
stage                  module                           reference
=====================  ===============================  ==========================================
L0 data acquisition    ``pfml.data.acquire``            0_Get_Additional_Data.py, 0_SP500_Subset.py
L2 panel preparation   ``pfml.models.prep``             Prepare_Data.py
L3 Barra risk model    ``pfml.models.risk``             Estimate Covariance Matrix.py
L4 PFML inputs         ``pfml.models.pfml_inputs``      PFML_Input_Data.py
L5 HP search           ``pfml.models.search``           PFML_Search_Coef.py, PFML_hp_reals.py
L6/L7 portfolio        ``pfml.models.portfolio``        PFML_aim_fun.py, PFML_hps.py, PFML_best_hps.py
orchestrator           ``pfml.pipeline``                Main.py
=====================  ===============================  ==========================================

Compute path: PyTorch-ROCm host orchestration over hand-written gfx950 HIP kernels
(``csrc/``, fp64 MFMA), RCCL over xGMI for multi-GPU (``pfml.parallel``), fp64 CPU oracle
for every op (``pfml.ops``).
"""
__version__ = "0.1.0"

from .config import Config, get_features, get_settings, pfml_feat_fun  # noqa: F401,E402
