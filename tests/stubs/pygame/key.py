def get_pressed():
    return [False] * 512
