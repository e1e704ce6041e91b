# Image for the job monitor (reference: kubernetes/jobmon/Dockerfile -- alpine + Go binary +
# kubectl). Here: the arena_amd package (jobmon is pure Python and imports no torch) + kubectl.
# The rendered jobmon Job runs `python -m arena_amd.runtime.jobmon` (charts.JOBMON_COMMAND); the
# `arena-jobmon` console script is installed too. Build from the repository root:
#   docker build -f deploy/jobmon.Dockerfile -t arena-amd/jobmon:latest .
FROM python:3.10-slim
ARG KUBECTL_VERSION=v1.29.0
ADD https://dl.k8s.io/release/${KUBECTL_VERSION}/bin/linux/amd64/kubectl /usr/local/bin/kubectl
RUN chmod +x /usr/local/bin/kubectl && pip install --no-cache-dir pyyaml
COPY arena_amd /opt/arena/arena_amd
ENV PYTHONPATH=/opt/arena ARENA_BACKEND=k8s
RUN printf '#!/bin/sh\nexec python -m arena_amd.runtime.jobmon "$@"\n' > /usr/local/bin/arena-jobmon \
    && chmod +x /usr/local/bin/arena-jobmon \
    && python -c "import arena_amd.runtime.jobmon, arena_amd.cluster.k8s"
ENTRYPOINT ["python", "-m", "arena_amd.runtime.jobmon"]
