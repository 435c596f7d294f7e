# COINSTAC-style computation image for MI355X (gfx950).  The base image provides ROCm + PyTorch;
# the gfx950 kernel library is compiled at image build time (hipcc cross-compiles, no GPU needed).
ARG BASE=rocm/pytorch:latest
FROM ${BASE}

WORKDIR /computation
COPY requirements.txt /computation/requirements.txt
RUN pip install --no-cache-dir -r requirements.txt

COPY . /computation
RUN PYTORCH_ROCM_ARCH=gfx950 python -m dinunet_implementations_amd.csrc.build --force

# one process per GPU site runs `python entry.py` under the COINSTAC runtime (or the stdio
# fallback of compat/coinstac.py); in-process multi-GPU training uses torchrun + run.py instead.
CMD ["python", "entry.py"]
