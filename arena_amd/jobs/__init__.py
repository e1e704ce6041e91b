"""L2 job model: submit specs, trainers (standalone / PS-worker / allreduce), GPU accounting."""
