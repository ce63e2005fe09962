"""Cell bit flags -- same names and values as safelife_game.CellTypes
(/root/reference/safelife/safelife_game.py:74-120)."""
import numpy as np


class CellTypes:
    alive_bit = 0
    agent_bit = 1
    pushable_bit = 2
    pullable_bit = 15
    destructible_bit = 3
    frozen_bit = 4
    preserving_bit = 5
    inhibiting_bit = 6
    spawning_bit = 7
    exit_bit = 8
    color_bit = 9

    alive = np.uint16(1 << alive_bit)
    agent = np.uint16(1 << agent_bit)
    pushable = np.uint16(1 << pushable_bit)
    pullable = np.uint16(1 << pullable_bit)
    destructible = np.uint16(1 << destructible_bit)
    frozen = np.uint16(1 << frozen_bit)
    preserving = np.uint16(1 << preserving_bit)
    inhibiting = np.uint16(1 << inhibiting_bit)
    spawning = np.uint16(1 << spawning_bit)
    exit = np.uint16(1 << exit_bit)
    color_r = np.uint16(1 << color_bit)
    color_g = np.uint16(1 << (color_bit + 1))
    color_b = np.uint16(1 << (color_bit + 2))

    empty = np.uint16(0)
    freezing = inhibiting | preserving
    player = agent | freezing | frozen | destructible
    wall = frozen
    movable = pushable | pullable
    crate = frozen | movable
    spawner = frozen | spawning | destructible
    hard_spawner = frozen | spawning
    level_exit = frozen | exit
    life = alive | destructible
    colors = (color_r, color_g, color_b)
    rainbow_color = color_r | color_g | color_b
    ice_cube = frozen | freezing | movable
    plant = frozen | alive | movable
    tree = frozen | alive
    fountain = preserving | frozen
    parasite = inhibiting | alive | pushable | frozen
    weed = preserving | alive | pushable | frozen
    powers = alive | freezing | spawning
