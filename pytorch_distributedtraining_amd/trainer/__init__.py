"""Training facade (Stoke-equivalent) and its configuration objects."""
from .configs import (AMPConfig, ClipGradConfig, ClipGradNormConfig, DDPConfig, DeepspeedConfig, DeepspeedZeROConfig,
                      DistributedOptions, FairscaleFSDPConfig, FairscaleOSSConfig, FairscaleSDDPConfig, FP16Options,
                      FSDPConfig, OSSConfig, SDDPConfig, StokeOptimizer)
from .status import StatusError, TrainerStatus
from .stoke import Stoke, SyncedLoss, Trainer

__all__ = ["AMPConfig", "ClipGradConfig", "ClipGradNormConfig", "DDPConfig", "DeepspeedConfig", "DeepspeedZeROConfig",
           "DistributedOptions", "FairscaleFSDPConfig", "FairscaleOSSConfig", "FairscaleSDDPConfig", "FP16Options",
           "FSDPConfig", "OSSConfig", "SDDPConfig", "StokeOptimizer", "StatusError", "TrainerStatus", "Stoke",
           "SyncedLoss", "Trainer"]
