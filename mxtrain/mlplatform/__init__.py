"""ML-platform services of the reference (charts/ml-platform/*, Kubeflow + Istio/Dex) for one node."""
