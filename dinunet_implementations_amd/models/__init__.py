"""Model families: FreeSurfer MLP (``MSANNet``) and the ICA bi-LSTM (``ICALstm``)."""
from .fs import MSANNet
from .ica import ICALstm, LSTM, LSTMCell

__all__ = ["MSANNet", "ICALstm", "LSTM", "LSTMCell"]
