"""model_2 plugin module (reference: model_2/model.py)."""
