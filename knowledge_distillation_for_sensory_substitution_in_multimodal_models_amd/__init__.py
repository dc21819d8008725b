"""MI355X-native (gfx950) online knowledge-distillation step.

Drop-in for the hot path of
shayekh00/Knowledge_Distillation_for_Sensory_Substitution_in_Multimodal_Models:
`OnlineKnowledgeDistillationLLavaOneVision.training_step` (RGB LLaVA-OneVision-7B
teacher -> depth LLaVA-OneVision-0.5B student), with every FLOP of the step in
hand-written HIP kernels behind the C-ABI library libkdstep.so (include/kdstep.h).
"""
__version__ = "0.1.0"
