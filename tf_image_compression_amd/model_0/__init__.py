"""model_0 plugin module (reference: model_0/model.py)."""
