class Error(Exception):
    """gym.error.Error"""
