"""dinunet_implementations_amd — MI355X-native decentralized neural-network trainer.

Same capabilities as trendscenter/dinunet_implementations (+ its coinstac-dinunet runtime):
FreeSurfer MLP and ICA bi-LSTM learners trained across sites with dSGD / rank-dAD / PowerSGD,
re-designed for MI355X: one site per GPU, RCCL collectives over xGMI, hand-written gfx950 HIP
kernels for the hot ops, HIP graphs for the launch-bound step.
"""
__version__ = "0.1.0"
