# Image for the allreduce job monitor (reference: kubernetes/jobmon/Dockerfile -- alpine + Go
# binary + kubectl). Here: the arena_amd package (pure Python for jobmon) + kubectl, run as
#   python -m arena_amd.runtime.jobmon   with NAMESPACE / JOBNAME / STATEFULSETNAME env.
FROM python:3.10-slim
ARG KUBECTL_VERSION=v1.29.0
ADD https://dl.k8s.io/release/${KUBECTL_VERSION}/bin/linux/amd64/kubectl /usr/local/bin/kubectl
RUN chmod +x /usr/local/bin/kubectl && pip install --no-cache-dir pyyaml
COPY arena_amd /opt/arena/arena_amd
ENV PYTHONPATH=/opt/arena ARENA_BACKEND=k8s
ENTRYPOINT ["python", "-m", "arena_amd.runtime.jobmon"]
