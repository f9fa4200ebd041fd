"""Dynamic plans on the host: the planner's routing keys and input streams
(utils/SiddhiExecutionPlanner.java:76-189, router/AddRouteOperator.java:
159-175) and the control-event classes (control/*.java).  No GPU needed."""
import pytest

import flink_siddhi as fs
from flink_siddhi.operator import (MetadataControlEvent, OperationControlEvent,
                                   plan_input_streams, plan_partition_keys,
                                   stream_definition_expression)

SCHEMA = [("id", "int"), ("name", "string"), ("price", "double"), ("timestamp", "long")]
DEFS = "".join(stream_definition_expression(s, SCHEMA)
               for s in ("inputStream1", "inputStream2", "inputStream3"))


def test_itcase_plans_partition_keys():
    # the four plans of SiddhiCEPITCase.testDynamicalStreamSimplePatternMatch (:484-505)
    assert plan_partition_keys(DEFS + "from inputStream1 select timestamp, id, name, price "
                               "insert into outputStream1;", "inputStream1") == []
    assert plan_partition_keys(DEFS + "from inputStream1 select id, timestamp, name, price "
                               "group by id insert into outputStream2;", "inputStream1") == ["id"]
    assert plan_partition_keys(DEFS + "from inputStream1 select name, timestamp, id, price "
                               "group by name insert into outputStream3;", "inputStream1") == ["name"]
    p4 = DEFS + "from inputStream2 select timestamp, id, name, price group by name insert into outputStream4;"
    assert plan_partition_keys(p4, "inputStream2") == ["name"]
    assert plan_partition_keys(p4, "inputStream1") == []
    assert plan_input_streams(p4) == ["inputStream2"]


def test_group_by_without_aggregates_is_a_projection():
    fs.validate(DEFS + "from inputStream1 select id, name group by id, name insert into O;")
    assert plan_partition_keys(DEFS + "from inputStream1 select id, name group by id, name "
                               "insert into O;", "inputStream1") == ["id", "name"]


def test_incompatible_partitions_are_rejected():
    # retrievePartition (SiddhiExecutionPlanner.java:172-189) throws on two
    # different group-by lists for one stream
    plan = (DEFS + "from inputStream1 select id, sum(price) as s group by id insert into O1;"
            "from inputStream1 select name, sum(price) as s group by name insert into O2;")
    with pytest.raises(fs.SiddhiAppCreationException, match="incompatible"):
        plan_partition_keys(plan, "inputStream1")
    same = (DEFS + "from inputStream1 select id, sum(price) as s group by id insert into O1;"
            "from inputStream1 select id, count() as c group by id insert into O2;")
    assert plan_partition_keys(same, "inputStream1") == ["id"]


def test_pattern_plans_route_by_partition_attribute():
    plan = (DEFS + "partition with (id of inputStream1, id of inputStream2) begin "
            "from every s1=inputStream1[price > 0.5] -> s2=inputStream2[price < 0.3] within 1 sec "
            "select s1.id as id, s2.price as p insert into O; end;")
    assert plan_input_streams(plan) == ["inputStream1", "inputStream2"]
    assert plan_partition_keys(plan, "inputStream1") == ["id"]
    assert plan_partition_keys(plan, "inputStream2") == ["id"]
    assert plan_partition_keys(plan, "inputStream3") == []
    with pytest.raises(fs.UndefinedStreamException):
        plan_partition_keys(plan, "nope")


def test_control_event_builders():
    ev = (MetadataControlEvent.builder()
          .add_execution_plan("a", "from inputStream1 select id insert into O;")
          .add_execution_plan("from inputStream2 select id insert into O;")
          .update_execution_plan("b", "x").remove_execution_plan("c").build())
    assert "a" in ev.added and len(ev.added) == 2
    assert ev.updated == {"b": "x"} and ev.deleted == ["c"]
    assert len(MetadataControlEvent.next_execution_plan_id()) == 36
    e = OperationControlEvent.disable_query("a")
    assert e.action == OperationControlEvent.Action.DISABLE_QUERY and e.query_id == "a"
    assert OperationControlEvent.enable_query("a").action.name == "ENABLE_QUERY"
    assert ev.name() == "MetadataControlEvent"
